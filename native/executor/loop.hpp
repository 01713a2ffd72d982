// Single-threaded epoll reactor + C++20 coroutines for the native shard executor.
//
// One process per shard group, one thread, no locks: the same concurrency model as the Python
// executor's asyncio loop, without its per-await cost.  `Task<T>` is a lazy coroutine awaited by
// its parent (symmetric transfer), `spawn` detaches one, `when_all` joins several; sockets are
// registered edge-triggered and awaited through `readable`/`writable`; `sleep` uses a timer heap.
#pragma once

#include <sys/epoll.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <coroutine>
#include <cstdio>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <optional>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace ncc {

inline double now_s() {
    using namespace std::chrono;
    return duration_cast<duration<double>>(steady_clock::now().time_since_epoch()).count();
}

// Scratch for one read: a coroutine that reads into a local array carries the array in its frame (a 64 KiB
// frame is past the pooled allocator's largest class, so every read would malloc and free it — and glibc
// trims the heap top with brk on that free).  Reads copy out of here before their next suspension point.
constexpr size_t kReadScratch = 1 << 16;
inline char* read_scratch() {
    static thread_local char b[kReadScratch];
    return b;
}

// ------------------------------------------------------------------------------------ Task
template <class T>
class Task;

// Stack guard for symmetric transfer.  A finished task resumes its awaiter by symmetric transfer, which
// is a tail call only when the compiler makes it one: at -O0/-O1 or under ASan GCC emits a nested call, so
// a worker whose awaits keep completing synchronously (queue never empty, nothing to write) grows the
// stack without bound.  Past kMaxNest bytes below the loop's frame the continuation is posted to the
// loop instead, which unwinds the stack; release builds never get near it.
inline char* g_stack_base = nullptr;                  // set by Loop::run
inline void (*g_post)(std::coroutine_handle<>) = nullptr;  // Loop::post of the running loop
constexpr std::ptrdiff_t kMaxNest = 256 * 1024;

namespace detail {
struct FinalAwaiter {
    bool await_ready() noexcept { return false; }
    template <class P>
    std::coroutine_handle<> await_suspend(std::coroutine_handle<P> h) noexcept {
        auto c = h.promise().cont;
        if (!c) return std::noop_coroutine();
        char probe;
        if (g_stack_base != nullptr && g_post != nullptr && g_stack_base - &probe > kMaxNest) {
            g_post(c);
            return std::noop_coroutine();
        }
        return c;
    }
    void await_resume() noexcept {}
};
struct PromiseBase {
    std::coroutine_handle<> cont;
    std::exception_ptr exc;
    std::suspend_always initial_suspend() noexcept { return {}; }
    FinalAwaiter final_suspend() noexcept { return {}; }
    void unhandled_exception() { exc = std::current_exception(); }
};
}  // namespace detail

template <class T>
class [[nodiscard]] Task {
public:
    struct promise_type : detail::PromiseBase {
        std::optional<T> value;
        Task get_return_object() { return Task(std::coroutine_handle<promise_type>::from_promise(*this)); }
        void return_value(T v) { value.emplace(std::move(v)); }
    };
    Task() = default;
    explicit Task(std::coroutine_handle<promise_type> h) : h_(h) {}
    Task(Task&& o) noexcept : h_(std::exchange(o.h_, {})) {}
    Task& operator=(Task&& o) noexcept {
        if (this != &o) {
            if (h_) h_.destroy();
            h_ = std::exchange(o.h_, {});
        }
        return *this;
    }
    Task(const Task&) = delete;
    ~Task() {
        if (h_) h_.destroy();
    }
    bool await_ready() const noexcept { return false; }
    std::coroutine_handle<> await_suspend(std::coroutine_handle<> c) noexcept {
        h_.promise().cont = c;
        return h_;
    }
    T await_resume() {
        if (h_.promise().exc) std::rethrow_exception(h_.promise().exc);
        return std::move(*h_.promise().value);
    }

private:
    std::coroutine_handle<promise_type> h_;
};

template <>
class [[nodiscard]] Task<void> {
public:
    struct promise_type : detail::PromiseBase {
        Task get_return_object() { return Task(std::coroutine_handle<promise_type>::from_promise(*this)); }
        void return_void() {}
    };
    Task() = default;
    explicit Task(std::coroutine_handle<promise_type> h) : h_(h) {}
    Task(Task&& o) noexcept : h_(std::exchange(o.h_, {})) {}
    Task& operator=(Task&& o) noexcept {
        if (this != &o) {
            if (h_) h_.destroy();
            h_ = std::exchange(o.h_, {});
        }
        return *this;
    }
    Task(const Task&) = delete;
    ~Task() {
        if (h_) h_.destroy();
    }
    bool await_ready() const noexcept { return false; }
    std::coroutine_handle<> await_suspend(std::coroutine_handle<> c) noexcept {
        h_.promise().cont = c;
        return h_;
    }
    void await_resume() {
        if (h_.promise().exc) std::rethrow_exception(h_.promise().exc);
    }

private:
    std::coroutine_handle<promise_type> h_;
};

// ------------------------------------------------------------------------------------ Loop
inline void g_loop_post(std::coroutine_handle<> h);

class Loop {
public:
    Loop() {
        ep_ = epoll_create1(EPOLL_CLOEXEC);
        if (ep_ < 0) throw std::runtime_error("epoll_create1 failed");
    }
    ~Loop() { ::close(ep_); }

    struct FdState {
        std::coroutine_handle<> reader, writer;
        bool readable = false, writable = false;
    };
    // Per-descriptor state indexed by the descriptor itself (small ints): no hashing on the per-event path.
    // A pointer from find() is valid until the next add().
    class FdTable {
    public:
        FdState* find(int fd) {
            return fd >= 0 && static_cast<size_t>(fd) < live_.size() && live_[static_cast<size_t>(fd)]
                       ? &st_[static_cast<size_t>(fd)]
                       : nullptr;
        }
        const FdState* find(int fd) const { return const_cast<FdTable*>(this)->find(fd); }
        FdState& add(int fd) {
            size_t i = static_cast<size_t>(fd);
            if (i >= st_.size()) {
                st_.resize(i * 2 + 16);
                live_.resize(i * 2 + 16, 0);
            }
            st_[i] = FdState{};
            live_[i] = 1;
            return st_[i];
        }
        void erase(int fd) {
            if (find(fd) == nullptr) return;
            st_[static_cast<size_t>(fd)] = FdState{};
            live_[static_cast<size_t>(fd)] = 0;
        }

    private:
        std::vector<FdState> st_;
        std::vector<uint8_t> live_;
    };

    void add_fd(int fd) {
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLOUT | EPOLLET | EPOLLRDHUP;
        ev.data.fd = fd;
        fds_.add(fd);
        if (epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev) != 0) throw std::runtime_error("epoll_ctl ADD failed");
    }
    void del_fd(int fd) {
        epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr);
        if (FdState* st = fds_.find(fd)) {
            // wake anyone still parked on the fd: their next syscall fails and raises
            if (st->reader) {
                post(st->reader);
                --parked_readers_;
            }
            if (st->writer) post(st->writer);
            fds_.erase(fd);
        }
    }

    struct IoAwait {
        Loop* loop;
        int fd;
        bool write;
        bool await_ready() {
            FdState* st = loop->fds_.find(fd);
            if (st == nullptr) return true;
            bool& flag = write ? st->writable : st->readable;
            if (flag) {
                flag = false;  // consumed: the caller retries its syscall
                return true;
            }
            return false;
        }
        void await_suspend(std::coroutine_handle<> h) {
            FdState* st = loop->fds_.find(fd);
            if (st == nullptr) {  // gone since await_ready: resume at once, the next syscall fails
                loop->post(h);
                return;
            }
            (write ? st->writer : st->reader) = h;
            if (!write) ++loop->parked_readers_;
        }
        void await_resume() {}
    };
    // Await the socket becoming readable/writable after a syscall returned EAGAIN (edge-triggered).
    IoAwait readable(int fd) { return IoAwait{this, fd, false}; }
    // Has an edge been reported for `fd` since it was last consumed?  (A reader whose last recv drained the
    // socket can wait for the next edge without first trying a recv that would return EAGAIN: every new
    // arrival of data raises an edge.)  Unknown descriptors count as readable: the next syscall fails.
    bool readable_now(int fd) const {
        const FdState* st = fds_.find(fd);
        return st == nullptr || st->readable;
    }
    IoAwait writable(int fd) { return IoAwait{this, fd, true}; }

    struct SleepAwait {
        Loop* loop;
        double until;
        bool await_ready() { return until <= now_s(); }
        void await_suspend(std::coroutine_handle<> h) { loop->timers_.push(Timer{until, loop->seq_++, h, {}}); }
        void await_resume() {}
    };
    SleepAwait sleep(double seconds) { return SleepAwait{this, now_s() + seconds}; }
    // Run `fn` on the loop at (or after) time `at`.
    void call_at(double at, std::function<void()> fn) { timers_.push(Timer{at, seq_++, {}, std::move(fn)}); }
    // epoll_wait returns so far (idle-loop diagnostics: an executor with nothing to do must not wake up)
    uint64_t wakeups() const { return wakeups_; }
    uint64_t coalesced() const { return coalesced_; }
    // Software interrupt coalescing (see run()): after a wake-up with few events while at least `min_parked`
    // readers wait, sleep `ns` before collecting the rest; 0 = off.
    void set_coalesce(long ns, int min_parked) {
        coalesce_ns_ = ns;
        coalesce_min_parked_ = min_parked;
    }

    void post(std::coroutine_handle<> h) { ready_.push_back(h); }
    void call_soon(std::function<void()> fn) { calls_.push_back(std::move(fn)); }
    void stop() { stopped_ = true; }
    bool stopped() const { return stopped_; }

    void run() {
        char base;
        g_stack_base = &base;
        g_post = &g_loop_post;
        epoll_event evs[256];
        while (!stopped_) {
            while (!ready_.empty() || !calls_.empty()) {
                while (!ready_.empty()) {
                    auto h = ready_.front();
                    ready_.pop_front();
                    h.resume();
                }
                while (!calls_.empty()) {
                    auto fn = std::move(calls_.front());
                    calls_.pop_front();
                    fn();
                }
                if (stopped_) return;
            }
            int timeout_ms = -1;
            double now = now_s();
            if (!timers_.empty()) {
                double dt = timers_.top().at - now;
                timeout_ms = dt <= 0 ? 0 : static_cast<int>(dt * 1000.0) + 1;
            }
            int n = epoll_wait(ep_, evs, 256, timeout_ms);
            ++wakeups_;
            if (n < 0 && errno != EINTR) throw std::runtime_error("epoll_wait failed");
            if (n > 0 && n < kCoalesceBelow && coalesce_ns_ > 0 && parked_readers_ >= coalesce_min_parked_) {
                // Under load (many requests awaiting their answers) a wake-up for one or two events is mostly
                // syscall and scheduler cost: let the answers that are on their way arrive, then take every
                // ready event in one more non-blocking call (software interrupt coalescing)
                timespec ts{0, coalesce_ns_};
                nanosleep(&ts, nullptr);
                int m = epoll_wait(ep_, evs + n, 256 - n, 0);
                if (m > 0) n += m;
                ++coalesced_;
            }
            for (int i = 0; i < n; ++i) {
                FdState* sp = fds_.find(evs[i].data.fd);
                if (sp == nullptr) continue;
                uint32_t e = evs[i].events;
                FdState& st = *sp;
                if (e & (EPOLLIN | EPOLLHUP | EPOLLERR | EPOLLRDHUP)) {
                    st.readable = true;
                    if (st.reader) {
                        auto h = std::exchange(st.reader, {});
                        st.readable = false;
                        ready_.push_back(h);
                        --parked_readers_;
                    }
                }
                if (e & (EPOLLOUT | EPOLLHUP | EPOLLERR)) {
                    st.writable = true;
                    if (st.writer) {
                        auto h = std::exchange(st.writer, {});
                        st.writable = false;
                        ready_.push_back(h);
                    }
                }
            }
            now = now_s();
            while (!timers_.empty() && timers_.top().at <= now) {
                const Timer& t = timers_.top();
                if (t.h)
                    ready_.push_back(t.h);
                else
                    calls_.push_back(t.fn);
                timers_.pop();
            }
        }
    }

private:
    struct Timer {
        double at;
        uint64_t seq;
        std::coroutine_handle<> h;  // resumed at `at`; or, when null,
        std::function<void()> fn;   // called at `at`
        bool operator>(const Timer& o) const { return at != o.at ? at > o.at : seq > o.seq; }
    };
    int ep_;
    bool stopped_ = false;
    uint64_t seq_ = 0;
    uint64_t wakeups_ = 0;
    uint64_t coalesced_ = 0;
    long coalesce_ns_ = 0;
    int coalesce_min_parked_ = 32;
    int parked_readers_ = 0;  // coroutines waiting for a descriptor to become readable
    static constexpr int kCoalesceBelow = 4;
    FdTable fds_;
    std::deque<std::coroutine_handle<>> ready_;
    std::deque<std::function<void()>> calls_;
    std::priority_queue<Timer, std::vector<Timer>, std::greater<Timer>> timers_;
};

inline Loop* g_loop = nullptr;
inline Loop& loop() { return *g_loop; }
inline void g_loop_post(std::coroutine_handle<> h) { g_loop->post(h); }

// ------------------------------------------------------------------------------------ Event
// Level-triggered flag with waiters (asyncio.Event), optionally with a deadline (`wait_for`).
class Event {
public:
    bool is_set() const { return set_; }
    void set() {
        set_ = true;
        for (auto h : waiters_) loop().post(h);
        waiters_.clear();
        for (auto& w : timed_) w->fire(true);
        timed_.clear();
    }
    void clear() { set_ = false; }
    struct Await {
        Event* ev;
        bool await_ready() { return ev->set_; }
        void await_suspend(std::coroutine_handle<> h) { ev->waiters_.push_back(h); }
        void await_resume() {}
    };
    Await wait() { return Await{this}; }

    // One waiter with a deadline: resumed once, by whichever comes first — set() (result true) or the
    // deadline timer (false).  The timer holds the node until it fires, so nothing dangles either way.
    struct TimedWaiter {
        std::coroutine_handle<> h;
        bool done = false, result = false;
        void fire(bool r) {
            if (done) return;
            done = true;
            result = r;
            loop().post(h);
        }
    };
    struct TimedAwait {
        Event* ev;
        double timeout;
        std::shared_ptr<TimedWaiter> node = std::make_shared<TimedWaiter>();
        bool await_ready() { return ev->set_ || timeout <= 0; }
        void await_suspend(std::coroutine_handle<> h) {
            node->h = h;
            ev->timed_.push_back(node);
            loop().call_at(now_s() + timeout, [n = node] { n->fire(false); });
        }
        bool await_resume() { return ev->set_ || node->result; }
    };
    // co_await ev.wait_for(seconds) -> whether the event is set (false: the deadline passed first).  No
    // polling: the waiter sleeps until set() or its single deadline timer.
    TimedAwait wait_for(double timeout) { return TimedAwait{this, timeout}; }

private:
    bool set_ = false;
    std::vector<std::coroutine_handle<>> waiters_;
    std::vector<std::shared_ptr<TimedWaiter>> timed_;
};

// ------------------------------------------------------------------------------------ spawn / when_all
struct Detached {
    struct promise_type {
        Detached get_return_object() { return {}; }
        std::suspend_never initial_suspend() noexcept { return {}; }
        std::suspend_never final_suspend() noexcept { return {}; }
        void return_void() {}
        void unhandled_exception() { std::terminate(); }
    };
};

inline Detached spawn_impl(Task<void> t, const char* what) {
    try {
        co_await t;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "{\"level\":\"error\",\"msg\":\"%s task failed: %s\"}\n", what, e.what());
    }
}
inline void spawn(Task<void> t, const char* what = "background") { spawn_impl(std::move(t), what); }

namespace detail {
struct JoinState {
    size_t left = 0;
    Event done;
    std::vector<std::exception_ptr> errs;
};
inline Detached join_one(Task<void> t, std::shared_ptr<JoinState> st, size_t i) {
    try {
        co_await t;
    } catch (...) {
        st->errs[i] = std::current_exception();
    }
    if (--st->left == 0) st->done.set();
}
}  // namespace detail

// Run every task concurrently; returns one exception_ptr per task (null on success).
inline Task<std::vector<std::exception_ptr>> when_all(std::vector<Task<void>> tasks) {
    std::vector<std::exception_ptr> out(tasks.size());
    if (tasks.empty()) co_return out;
    if (tasks.size() == 1) {
        try {
            co_await tasks[0];
        } catch (...) {
            out[0] = std::current_exception();
        }
        co_return out;
    }
    auto st = std::make_shared<detail::JoinState>();
    st->left = tasks.size();
    st->errs.resize(tasks.size());
    for (size_t i = 0; i < tasks.size(); ++i) detail::join_one(std::move(tasks[i]), st, i);
    co_await st->done.wait();
    co_return std::move(st->errs);
}

}  // namespace ncc
