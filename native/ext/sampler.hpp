// native/ext/sampler.hpp — where the Python processes' time inside this extension goes.
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
//
// ncc/sampler.py's SIGPROF profile charges a native call to the Python line that made it, so the coordinator's
// biggest lines (the owner filter, the slim template decode, the relay index, the inline finish) are each one
// opaque call.  With NCC_NATIVE_SAMPLE set, `native_sample_start` installs a SIGPROF handler in front of
// Python's: each tick records the interrupted instruction address and the word on top of the stack, then hands
// the signal on (the Python-level profile keeps working), and `native_sample_dump` writes them with the
// executable mappings in the C++ executor's format, so scripts/executor_profile.py symbolizes them
// (`--binary ncc/_native...so`).
#pragma once
// (signal.h, sys/time.h, ucontext.h: included at the top of native/ncc_native.cpp, outside the namespace)

constexpr size_t kNativeMaxSamples = 1 << 18;
static uintptr_t* g_nsamples_buf = nullptr;  // pairs: pc, top-of-stack word
static volatile size_t g_nsamples_n = 0;
static struct sigaction g_nsamples_prev {};

#if defined(__x86_64__)
static void native_on_sigprof(int sig, siginfo_t* si, void* ucv) {
    auto* uc = static_cast<ucontext_t*>(ucv);
    size_t n = g_nsamples_n;
    if (g_nsamples_buf != nullptr && n < kNativeMaxSamples) {
        g_nsamples_buf[2 * n] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
        g_nsamples_buf[2 * n + 1] = *reinterpret_cast<const uintptr_t*>(uc->uc_mcontext.gregs[REG_RSP]);
        g_nsamples_n = n + 1;
    }
    if (g_nsamples_prev.sa_flags & SA_SIGINFO) {
        if (g_nsamples_prev.sa_sigaction != nullptr) g_nsamples_prev.sa_sigaction(sig, si, ucv);
    } else if (g_nsamples_prev.sa_handler != SIG_DFL && g_nsamples_prev.sa_handler != SIG_IGN &&
               g_nsamples_prev.sa_handler != nullptr) {
        g_nsamples_prev.sa_handler(sig);
    }
}
#endif

// Starts sampling; `us`: the ITIMER_PROF interval (kept when a timer already runs: ncc/sampler.py's).
bool native_sample_start(long us) {
#if !defined(__x86_64__)
    return false;
#else
    if (g_nsamples_buf == nullptr) g_nsamples_buf = new uintptr_t[2 * kNativeMaxSamples];
    struct sigaction sa {};
    sa.sa_sigaction = native_on_sigprof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    struct sigaction prev {};
    sigaction(SIGPROF, &sa, &prev);
    if (prev.sa_sigaction != native_on_sigprof) g_nsamples_prev = prev;  // never chain to ourselves
    struct itimerval cur {};
    getitimer(ITIMER_PROF, &cur);
    if (cur.it_interval.tv_sec == 0 && cur.it_interval.tv_usec == 0) {
        us = std::max(50L, us);
        struct itimerval it {};
        it.it_interval.tv_sec = us / 1000000;
        it.it_interval.tv_usec = us % 1000000;
        it.it_value = it.it_interval;
        setitimer(ITIMER_PROF, &it, nullptr);
    }
    return true;
#endif
}

// Writes the samples to `path` ("# map" lines of the executable mappings, then "pc tos" per sample).
size_t native_sample_dump(const std::string& path) {
    if (g_nsamples_buf == nullptr) return 0;
    FILE* f = std::fopen(path.c_str(), "w");
    if (f == nullptr) return 0;
    if (FILE* maps = std::fopen("/proc/self/maps", "r")) {
        char line[4096];
        while (std::fgets(line, sizeof line, maps) != nullptr)
            if (std::strstr(line, " r-xp ") != nullptr) std::fprintf(f, "# map %s", line);
        std::fclose(maps);
    }
    size_t n = g_nsamples_n;
    for (size_t i = 0; i < n; ++i)
        std::fprintf(f, "%zx %zx\n", static_cast<size_t>(g_nsamples_buf[2 * i]),
                     static_cast<size_t>(g_nsamples_buf[2 * i + 1]));
    std::fclose(f);
    return n;
}
