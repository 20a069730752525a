"""A tripped watchdog is an error the caller cannot miss, and
the blocking shims wait only for their own work.

The bounded inter-workgroup waits (k_final_ipn of NTT_PLAN_IN_PLACE plans, k_fused3 / k_fused3b of
NTT_PLAN_SINGLE_LAUNCH plans) give up after ntt_plan_set_watchdog's poll limit.  With the limit at 0
(the test hook) the waits that are not already satisfied give up at once: the workgroup skips its
stores, the plan's host-mapped report word is set, and the NEXT call on the plan returns
NTT_ERR_DEVICE without any device query.  ntt_plan_device_status reports bit 0 and clears the
report; with the default limit restored the plan is correct again.  The reference asserts instead
(GZKP-NTT.cu:1527)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _fresh(plan, seed):
    return plan.fill(plan.empty(), "random", seed=seed)


@pytest.mark.parametrize("flag,log_n,direction", [("in_place", 22, "forward"), ("in_place", 22, "inverse"),
                                                   ("in_place", 20, "forward"), ("single", 20, "forward"),
                                                   ("single", 20, "inverse"), ("dataflow", 20, "forward"),
                                                   ("ip_single", 20, "forward"), ("ip_single", 19, "inverse")])
def test_watchdog_trip_is_reported_and_plan_recovers(flag, log_n, direction, monkeypatch):
    from ntt_amd import lib as L
    from ntt_amd.ntt import NTTPlan
    if flag in ("single", "dataflow"):  # the single-launch form: grid barriers (1, default) or dataflow (0)
        monkeypatch.setenv("NTT_FUSED_MODE", "1" if flag == "single" else "0")
    ref = NTTPlan(1, log_n, 4)
    # ip_single: the in-place single launch (three grid barriers, k_fused3bi)
    pl = NTTPlan(1, log_n, 4, in_place=flag in ("in_place", "ip_single"), single_launch=flag != "in_place")
    run = (lambda p, t: p.forward(t)) if direction == "forward" else (lambda p, t: p.inverse(t))
    x = _fresh(ref, 3)
    want = x.clone()
    run(ref, want)
    got = x.clone()
    run(pl, got)  # healthy first (builds the fused / in-place schedule)
    torch.cuda.synchronize()
    assert pl.device_status() == 0 and torch.equal(got, want)

    pl.set_watchdog(0)  # every wait that is not already satisfied gives up at once
    bad = x.clone()
    run(pl, bad)  # enqueued fine: the trip is only known once the kernel has run
    torch.cuda.synchronize()
    with pytest.raises(L.NTTError) as ei:  # the next call refuses, with no device query
        run(pl, x.clone())
    assert ei.value.status == L.NTT_ERR_DEVICE
    with pytest.raises(L.NTTError) as ei:
        pl.forward(x.clone())
    assert ei.value.status == L.NTT_ERR_DEVICE
    assert not torch.equal(bad, want)  # the tripped call's output is wrong (and was reported)
    assert pl.device_status() & 1  # reported, then cleared

    pl.set_watchdog()  # default limit: the plan is usable again and correct
    again = x.clone()
    run(pl, again)
    torch.cuda.synchronize()
    assert torch.equal(again, want)
    assert pl.device_status() == 0


def test_blocking_shim_does_not_wait_for_other_streams():
    """SSIP / NTT_GZKP_256 wait on an event after their own launches (GZKP-NTT.cu:1547), not on the
    whole device: work queued on another (non-blocking) stream is still running when the shim
    returns.  The side stream starts with a ~2 s spin kernel, far longer than any shim call, so the
    check needs no wall-clock bound."""
    from ntt_amd.ntt import NTTPlan, SSIP
    big = NTTPlan(1, 24, 4)
    y = _fresh(big, 5)
    x = torch.arange(1 << 12, dtype=torch.int64, device="cuda:0")
    SSIP(x.clone(), 3, 12)  # warm the shim's cached plan
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(int(4e9))  # ~2 s of clock cycles: the side stream is busy long after the shim
        for _ in range(300):  # ~0.45 s of transforms
            big.forward(y, stream=side)
    out = SSIP(x.clone(), 3, 12)
    still_running = not side.query()
    side.synchronize()
    assert still_running
    x2 = x.clone()
    SSIP(x2, 3, 12)
    assert torch.equal(out, x2)
