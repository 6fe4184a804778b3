"""The keyBy exchange's bounded wait (flink_amd/csrc/gw_wait.h), on the CPU.

gw_exchange_batch / gw_exchange_min_watermark never block in hipStreamSynchronize behind an
RCCL collective: they poll the stream, ncclCommGetAsyncError and a deadline, and abort the
communicator on an error or expiry (a failed channel fails the task in the reference:
KeyGroupStreamPartitioner.java:55-64 writes into channels whose failures fail the task;
StatusWatermarkValve.java:153-185 never waits on a dead input).  The policy is header-only
and compiled here with g++ against injected stream states, asynchronous errors and a fake
clock, so every exit of the wait is exercised without a GPU or a second rank."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DONE, STREAM_ERROR, COMM_ERROR, TIMEOUT = 0, 1, 2, 3


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("wait") / "wait_policy")
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "flink_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "wait_policy.cpp"), "-o", exe, "-pthread"], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=60).stdout
    return {ln.split()[0]: [int(x) for x in ln.split()[1:]] for ln in out.splitlines()}


def test_completion_ends_the_wait(results):
    r, polls, relaxes, _ = results["done"]
    assert (r, polls, relaxes) == (DONE, 5, 4)


def test_never_completing_stream_times_out(results):
    r, polls, _, clock = results["timeout"]
    assert r == TIMEOUT
    # one clock read at the start and one per poll, 1 ms each: expiry at the 50 ms deadline
    assert 49 <= polls <= 51 and clock >= 50_000_000


def test_async_communicator_error_aborts(results):
    assert results["comm"][:2] == [COMM_ERROR, 7]


def test_stream_error_aborts(results):
    assert results["stream"][:2] == [STREAM_ERROR, 3]


def test_no_deadline_waits_until_an_error(results):
    assert results["nodeadline_comm"][:2] == [COMM_ERROR, 10000]


def test_completion_is_checked_before_errors(results):
    assert results["done_first"][:2] == [DONE, 1]


def test_real_clock_deadline(results):
    r, polls, ms = results["real"]
    assert r == TIMEOUT and 30 <= ms < 5000 and polls > 1
