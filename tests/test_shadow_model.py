"""ShadowComm (rank 0 of a p-rank job alone on one device, bench/bench_emulate.py) and its
communication-cost model: the ring broadcast costs lat + bytes / bw on one link; the direct
broadcast (Comm::bcast_direct) is modelled as its two point-to-point rounds, each lat + the busiest
link's bytes / bw.  On the host device the modelled cost is only accounted (no spin kernels), which
is what these tests check."""
import pytest

from mpi_jordan_crazy_acceleration_amd import load_native


def _solve(C, p, direct, monkeypatch, n=2048, m=64, bw=50.0, lat=20.0):
    monkeypatch.setenv("GJ_BCAST", "direct" if direct else "ring")
    comm = C.shadow_comm(p, bw, lat, 16, direct=direct)
    eng = C.Engine(C.host_device(4), comm, n, m, "fp64")
    eng.generate("random", 1)
    st = eng.solve()
    return eng, st, C.shadow_modelled_us(comm), comm


@pytest.mark.parametrize("p", [4, 8])
def test_direct_broadcast_is_modelled(p, monkeypatch):
    C = load_native()
    eng_r, st_r, us_r, comm_r = _solve(C, p, False, monkeypatch)
    eng_d, st_d, us_d, comm_d = _solve(C, p, True, monkeypatch)
    assert st_r["status"] == 0 and st_d["status"] == 0
    assert eng_r.layout["bcast"] == "ring" and eng_d.layout["bcast"] == "direct"
    assert "direct broadcast" in comm_d.describe()
    # row segments of m x chunk width (>= 64 KiB) go direct: per byte 2/(p-1) of the ring's link
    # time plus one more latency per message
    assert us_d != us_r and us_r > 0 and us_d > 0


def test_ring_only_shadow_cannot_go_direct(monkeypatch):
    C = load_native()
    monkeypatch.setenv("GJ_BCAST", "direct")
    comm = C.shadow_comm(4, 50.0, 20.0, 16)  # direct=False: no point-to-point path modelled
    eng = C.Engine(C.host_device(2), comm, 512, 32, "fp64")
    assert eng.layout["bcast"] == "ring"
    assert "no point-to-point" in comm.bcast_report()


def test_p2p_cost_is_per_link(monkeypatch):
    # a large direct broadcast: the model must charge ~2 * bytes / (p - 1) / bw, not bytes / bw
    C = load_native()
    monkeypatch.setenv("GJ_BCAST", "direct")
    p, bw, lat = 8, 50.0, 0.0
    comm = C.shadow_comm(p, bw, lat, 16, direct=True)
    eng = C.Engine(C.host_device(2), comm, 4096, 128, "fp64", depth=1)
    before = C.shadow_modelled_us(comm)
    assert eng.layout["bcast"] == "direct"
    nbytes = 64 << 20
    C.shadow_bcast_probe(comm, nbytes, 1)
    modelled = C.shadow_modelled_us(comm) - before
    slice_us = (nbytes / (p - 1)) / (bw * 1e3)
    assert modelled == pytest.approx(2 * slice_us, rel=0.02)


@pytest.mark.parametrize("pivot", ["block-min-inv-norm", "partial"])
def test_shadow_synthetic_peers_win_under_both_rules(pivot):
    """The emulated peers' records must win at every step t with t % p != 0 under either pivot rule
    (Partial scores are -max|W| < 0, so a synthetic score of 0 would lose to rank 0's own block; ADVICE
    r3), and the step comes from the engine (a partial fallback's second exchange repeats a step)."""
    C = load_native()
    p, n, m = 4, 512, 32
    comm = C.shadow_comm(p, 0.0, 0.0, 16)
    eng = C.Engine(C.host_device(2), comm, n, m, "fp64", pivot=pivot)
    eng.generate("random", 1)
    st = eng.solve()
    assert st["status"] == 0
    piv = st["pivots"]
    assert all(piv[t] == t for t in range(len(piv)) if t % p != 0), piv
    assert all(piv[t] % p == 0 for t in range(len(piv)) if t % p == 0), piv
