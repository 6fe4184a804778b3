"""gw_exchange_plan (include/gpuwin.h), the per-peer send / receive plan gw_exchange_batch runs
after its count all-to-all, at P = 2..8 ranks on the CPU: every rank's plan from the messages
it sent and received must agree with every peer's (what q sends to r is what r receives from
q, at the offsets both computed), the receive columns hold the peers' records in rank order
(torch.distributed.all_to_all_single's layout, which the gloo rehearsal of tests/test_multirank.py
also checks against the plan with real point-to-point transfers), the watermark is the minimum
over the ranks (StatusWatermarkValve.inputWatermark, flink-runtime/.../watermarkstatus/
StatusWatermarkValve.java:153-185), and a rank passing other columns fails every rank before
any transfer (KeyGroupStreamPartitioner.selectChannel routing itself: tests/test_multirank.py)."""
import numpy as np
import pytest

from flink_amd import _native as N


def messages(counts, wms, masks, packed=None):
    """msg[r] (sent by r) and rmsg[r] (received by r): (records, watermark, mask, packed
    records) per peer."""
    P = len(wms)
    pk = np.zeros_like(counts) if packed is None else packed
    sent = [np.array([[counts[r][q], wms[r], masks[r], pk[r][q]] for q in range(P)], np.int64).ravel()
            for r in range(P)]
    recv = [np.array([[counts[q][r], wms[q], masks[q], pk[q][r]] for q in range(P)], np.int64).ravel()
            for r in range(P)]
    return sent, recv


@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8])
def test_plans_agree_across_ranks_and_lay_out_by_rank(P):
    rng = np.random.default_rng(P)
    counts = rng.integers(0, 1000, (P, P))
    counts[rng.random((P, P)) < 0.2] = 0  # peers without records for a rank
    wms = rng.integers(-(1 << 40), 1 << 40, P)
    sent, recv = messages(counts, wms, [1] * P)
    # each rank's owner-partitioned columns: record i for peer q tagged (r, q, i)
    send_cols = [np.concatenate([np.array([r * 1_000_000 + q * 1000 + i for i in range(counts[r][q])], np.int64)
                                 for q in range(P)]) for r in range(P)]
    plans = [N.exchange_plan(sent[r], recv[r], 1, int(wms[r])) for r in range(P)]
    for r, ((so, sc, ro, rc), total, wmin) in enumerate(plans):
        assert total == counts[:, r].sum()
        assert wmin == wms.min()
        assert list(sc) == list(counts[r]) and list(rc) == list(counts[:, r])
        assert list(so) == list(np.concatenate([[0], np.cumsum(counts[r])[:-1]]))
        assert list(ro) == list(np.concatenate([[0], np.cumsum(counts[:, r])[:-1]]))
        # receive columns filled by every peer's send, at the offsets both sides computed
        buf = np.full(total, -1, np.int64)
        for q in range(P):
            (qso, qsc, _, _), _, _ = plans[q]
            assert qsc[r] == rc[q]
            buf[ro[q]:ro[q] + rc[q]] = send_cols[q][qso[r]:qso[r] + qsc[r]]
        # all_to_all_single's layout: peer 0's records for r, then peer 1's, ...
        expect = np.concatenate([np.array([q * 1_000_000 + r * 1000 + i for i in range(counts[q][r])], np.int64)
                                 for q in range(P)])
        assert np.array_equal(buf, expect)


@pytest.mark.parametrize("P", [2, 5, 8])
def test_column_mismatch_fails_every_rank(P):
    counts = np.full((P, P), 3)
    masks = [1] * P
    masks[P - 1] = 3  # the last rank also ships key hashes
    sent, recv = messages(counts, np.zeros(P, np.int64), masks)
    for r in range(P):
        with pytest.raises(N.GpuWinError) as ei:
            N.exchange_plan(sent[r], recv[r], masks[r], 0)
        assert ei.value.code == N.GW_E_INVALID


def test_negative_counts_are_invalid():
    sent, recv = messages(np.array([[1, -2], [3, 4]]), np.zeros(2, np.int64), [1, 1])
    with pytest.raises(N.GpuWinError):
        N.exchange_plan(sent[0], recv[0], 1, 0)


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_packed_plans_agree_across_ranks(P):
    """gw_exchange_plan_packed: q's packed words go first in its send range, its other records
    follow; on the receiver the other records of all peers come first (rank order), then the
    peers' words in rank order -- what r receives from q is what q sent to r."""
    rng = np.random.default_rng(100 + P)
    counts = rng.integers(0, 600, (P, P))
    packed = (counts * rng.random((P, P))).astype(np.int64)
    packed[rng.random((P, P)) < 0.2] = 0
    sent, recv = messages(counts, np.zeros(P, np.int64), [5] * P, packed)
    for r in range(P):
        (so, sc, _, rc), total, _ = N.exchange_plan(sent[r], recv[r], 5, 0)
        (sp, rwo, rpo, rp), tw, tp = N.exchange_plan_packed(sent[r], recv[r])
        assert list(sp) == list(packed[r]) and list(rp) == list(packed[:, r])
        assert tw + tp == total and tp == packed[:, r].sum()
        assert list(rwo) == list(np.concatenate([[0], np.cumsum(counts[:, r] - packed[:, r])[:-1]]))
        assert list(rpo) == list(np.concatenate([[0], np.cumsum(packed[:, r])[:-1]]))
        for q in range(P):  # the sender's view of the same transfer
            (_, qsc, _, _), _, _ = N.exchange_plan(sent[q], recv[q], 5, 0)
            (qsp, _, _, _), _, _ = N.exchange_plan_packed(sent[q], recv[q])
            assert qsp[r] == rp[q] and qsc[r] - qsp[r] == rc[q] - rp[q]


def test_packed_count_above_records_is_invalid():
    sent, recv = messages(np.array([[4, 4], [4, 4]]), np.zeros(2, np.int64), [5, 5], np.array([[5, 0], [0, 0]]))
    with pytest.raises(N.GpuWinError):
        N.exchange_plan(sent[0], recv[0], 5, 0)
    with pytest.raises(N.GpuWinError):
        N.exchange_plan_packed(sent[0], recv[0])
