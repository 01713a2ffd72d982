// Test tool (never shipped): the executor's open-addressing map (native/executor/strmap.hpp) against
// std::unordered_map under random operations — inserts (operator[], emplace, try_emplace), finds of present and
// absent keys, erases by key and by iterator (also while iterating), clears, moves, growth past several
// rehashes and tombstone-only rehashes — comparing contents after every step batch.  Prints one JSON line and
// exits 1 on the first difference.  tests/test_executor_strmap.py runs it.
//
//   ncc-strmap-check [seed] [steps]
#include "../executor/strmap.hpp"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

int fail(const char* what, long step, const std::string& key) {
    std::printf("{\"ok\": false, \"what\": \"%s\", \"step\": %ld, \"key\": \"%s\"}\n", what, step, key.c_str());
    return 1;
}

// a value with a destructor, so leaks and double destruction show in the live count
struct Val {
    static long live;
    std::shared_ptr<int> p;
    Val() : p(std::make_shared<int>(0)) { ++live; }
    explicit Val(int v) : p(std::make_shared<int>(v)) { ++live; }
    Val(const Val& o) : p(o.p) { ++live; }
    Val(Val&& o) noexcept : p(std::move(o.p)) { ++live; }
    Val& operator=(const Val& o) = default;
    Val& operator=(Val&& o) noexcept = default;
    ~Val() { --live; }
    int get() const { return p ? *p : -1; }
};
long Val::live = 0;

}  // namespace

int main(int argc, char** argv) {
    unsigned seed = argc > 1 ? static_cast<unsigned>(std::atoi(argv[1])) : 1;
    long steps = argc > 2 ? std::atol(argv[2]) : 200000;
    std::mt19937 rnd(seed);
    {
        ncc::StrMap<Val> m;
        std::unordered_map<std::string, int> ref;
        long universe = 64;
        auto key = [&]() {
            // keys of every length class: short (SSO), 16-40 bytes (the executor's "namespace/name")
            long i = static_cast<long>(rnd() % static_cast<unsigned>(universe));
            std::string k = (i % 3 == 0) ? "k" + std::to_string(i) : "namespace-" + std::to_string(i % 7) + "/object-name-" + std::to_string(i);
            return k;
        };
        for (long step = 0; step < steps; ++step) {
            if (step % 20000 == 0) universe = 16 + static_cast<long>(rnd() % 6000);  // phases of growth and churn
            unsigned op = rnd() % 100;
            std::string k = key();
            int v = static_cast<int>(rnd() % 1000000);
            if (op < 25) {
                m[k] = Val(v);
                ref[k] = v;
            } else if (op < 35) {
                auto [it, fresh] = m.try_emplace(k, v);
                auto [rit, rfresh] = ref.try_emplace(k, v);
                if (fresh != rfresh || it->second.get() != rit->second || it->first != k) return fail("try_emplace", step, k);
            } else if (op < 42) {
                auto [it, fresh] = m.emplace(std::string(k), Val(v));
                auto [rit, rfresh] = ref.emplace(k, v);
                if (fresh != rfresh || it->second.get() != rit->second) return fail("emplace", step, k);
            } else if (op < 65) {
                auto it = m.find(k);
                auto rit = ref.find(k);
                if ((it == m.end()) != (rit == ref.end())) return fail("find", step, k);
                if (it != m.end() && (it->second.get() != rit->second || it->first != k)) return fail("find value", step, k);
                if (m.count(k) != ref.count(k)) return fail("count", step, k);
            } else if (op < 80) {
                if (m.erase(k) != ref.erase(k)) return fail("erase key", step, k);
            } else if (op < 85) {
                auto it = m.find(k);
                if (it != m.end()) {
                    m.erase(it);
                    ref.erase(k);
                }
            } else if (op < 88) {  // erase a random share while iterating
                unsigned every = 2 + rnd() % 4;
                unsigned n = 0;
                for (auto it = m.begin(); it != m.end();) {
                    if (++n % every == 0) {
                        ref.erase(it->first);
                        it = m.erase(it);
                    } else {
                        ++it;
                    }
                }
            } else if (op < 89) {
                ncc::StrMap<Val> other = std::move(m);
                if (!m.empty() || m.find(k) != m.end()) return fail("moved-from not empty", step, k);
                m = std::move(other);
            } else if (op == 89 && rnd() % 50 == 0) {
                m.clear();
                ref.clear();
            } else if (op < 92) {
                m.reserve(m.size() + rnd() % 2000);
            }
            if (m.size() != ref.size()) return fail("size", step, k);
            if (step % 997 == 0) {  // full comparison, both directions
                size_t seen = 0;
                for (const auto& kv : m) {
                    auto rit = ref.find(kv.first);
                    if (rit == ref.end() || rit->second != kv.second.get()) return fail("content", step, kv.first);
                    ++seen;
                }
                if (seen != ref.size()) return fail("iteration count", step, k);
                const auto& cm = m;
                for (const auto& kv : ref) {
                    auto it = cm.find(kv.first);
                    if (it == cm.end() || it->second.get() != kv.second) return fail("missing", step, kv.first);
                }
            }
        }
        if (Val::live != static_cast<long>(m.size())) return fail("live values", steps, std::to_string(Val::live));
    }
    if (Val::live != 0) return fail("leak", steps, std::to_string(Val::live));
    std::printf("{\"ok\": true, \"seed\": %u, \"steps\": %ld}\n", seed, steps);
    return 0;
}
