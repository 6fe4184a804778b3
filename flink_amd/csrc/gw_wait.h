// gw_wait.h — bounded wait for work queued behind an RCCL collective (gw_exchange.cpp).
//
// A failed network channel fails the task in the reference (KeyGroupStreamPartitioner /
// RecordWriter write into Netty channels whose errors surface as task failures; the
// watermark valve, StatusWatermarkValve.java:153-185, never waits on a dead input forever).
// An RCCL peer that dies or diverges instead leaves ncclAllToAll / ncclSend spinning on the
// GPU, and a plain hipStreamSynchronize behind it blocks the host for good.  The exchange
// therefore never blocks: it polls the stream, the communicator's asynchronous error and a
// deadline, and on expiry or error aborts the communicator (ncclCommAbort makes the kernels
// spinning on a dead peer return) and fails the call.
//
// Header-only and free of HIP / RCCL types so the policy is tested on the CPU with injected
// stubs (tests/test_exchange_wait.py compiles it with g++).
#pragma once
#include <chrono>
#include <cstdint>
#include <thread>

namespace gw {

enum class WaitResult { kDone = 0, kStreamError = 1, kCommError = 2, kTimeout = 3 };

// query():       0 done, 1 still running, 2 stream error
// async_error(): 0 none (or in progress), else the communicator failed
// now_ns():      a monotonic clock
// relax(k):      what the waiter does between polls (k: polls so far); spinning first keeps the
//                common ~10-50 us wait off the scheduler, then it yields / sleeps
// deadline_ns <= 0: no deadline (only errors end a wait that never completes)
template <class Query, class AsyncError, class Now, class Relax>
WaitResult poll_until_done(Query query, AsyncError async_error, Now now_ns, Relax relax, int64_t deadline_ns,
                           int64_t* polls = nullptr) {
    const int64_t t0 = now_ns();
    for (int64_t k = 0;; ++k) {
        if (polls) *polls = k + 1;
        const int q = query();
        if (q == 0) return WaitResult::kDone;
        if (q != 1) return WaitResult::kStreamError;
        if (async_error() != 0) return WaitResult::kCommError;
        if (deadline_ns > 0 && now_ns() - t0 >= deadline_ns) return WaitResult::kTimeout;
        relax(k);
    }
}

inline int64_t steady_now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// ~2k spins (tens of us), then yields, then 50-us sleeps
inline void relax_backoff(int64_t k) {
    if (k < 2048) return;
    if (k < 4096) { std::this_thread::yield(); return; }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
}

}  // namespace gw
