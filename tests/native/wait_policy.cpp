// CPU driver for gw_wait.h (tests/test_exchange_wait.py): the exchange's bounded wait with
// injected stream states, asynchronous communicator errors and a fake clock.
#include <cstdio>
#include <cstdlib>

#include "gw_wait.h"

using gw::WaitResult;

// scenario: done_at (-1 never), stream_err_at, comm_err_at, clock step per now() call (ns),
// deadline (ns)
static void run(const char* name, int64_t done_at, int64_t stream_err_at, int64_t comm_err_at, int64_t step_ns,
                int64_t deadline_ns) {
    int64_t polls_q = 0, clock = 0, relaxes = 0, polls = 0;
    auto query = [&] {
        ++polls_q;
        if (stream_err_at >= 0 && polls_q >= stream_err_at) return 2;
        return done_at >= 0 && polls_q >= done_at ? 0 : 1;
    };
    auto async_err = [&] { return comm_err_at >= 0 && polls_q >= comm_err_at ? 1 : 0; };
    auto now = [&] { clock += step_ns; return clock; };
    auto relax = [&](int64_t) { ++relaxes; };
    const WaitResult r = gw::poll_until_done(query, async_err, now, relax, deadline_ns, &polls);
    printf("%s %d %lld %lld %lld\n", name, (int)r, (long long)polls, (long long)relaxes, (long long)clock);
}

int main() {
    run("done", 5, -1, -1, 1000, 1000000);
    run("timeout", -1, -1, -1, 1000000, 50000000);  // 1 ms per clock read, 50 ms deadline
    run("comm", -1, -1, 7, 1000, 1000000000);
    run("stream", -1, 3, -1, 1000, 1000000000);
    run("nodeadline_comm", -1, -1, 10000, 1000000000, 0);  // no deadline: only the error ends it
    run("done_first", 1, -1, 1, 1000, 1000);  // completion wins over a late error flag
    // the real clock and backoff: a never-completing stream ends at a 30 ms deadline
    int64_t polls = 0;
    const int64_t t0 = gw::steady_now_ns();
    const WaitResult r = gw::poll_until_done([] { return 1; }, [] { return 0; }, gw::steady_now_ns,
                                             gw::relax_backoff, 30000000, &polls);
    printf("real %d %lld %lld\n", (int)r, (long long)polls, (long long)((gw::steady_now_ns() - t0) / 1000000));
    return 0;
}
