"""GPU: the library's own multi-rank exchange at R > 1 on one GPU, through the in-process
loopback transport (gpmdm_comm_init_loopback, test only).

RCCL refuses two ranks on one device, so on a one-GPU box the library's exchange
(gpmdm_pf_set_comm: pack -> all-gather on the library stream -> events -> rows read in
place; the uneven-shard staging + copy-down; the grouped collectives of
gpmdm_pf_propagate_multi) would otherwise only ever run with one rank.  The loopback
communicators stand in for RCCL's behind the same calls, with its completion semantics, so
those paths run here with R = 2, 4 and 8 ranks:

* ``GPMDM_PF(devices=[0] * R, transport='loopback')``: one thread drives every rank
  (gpmdm_pf_propagate_multi, grouped collectives);
* R filters of ``shard=(R, r)`` with ``set_comm(loopback[r])``, each stepped by a thread of
  its own on a stream of its own (gpmdm_pf_propagate: each rank blocks in the collective
  until every rank has joined, as ranks in separate processes do).

Every frame's read-outs and the final exported state must be bitwise the one-rank filter's
(the reference's replicated filter, gpmdm_pf.py:117-262; exchange point :194-213).
P = 10,007 gives uneven shards (the staging path); P = 10,008 with ``pad_rows`` forces it on
even shards."""
import threading

import numpy as np
import pytest
import torch

from conftest import product_model

pytestmark = pytest.mark.gpu

FRAMES = 4


@pytest.fixture(scope="module")
def m2(fx_config2):
    return product_model(fx_config2)


def _z(m, k):
    return np.ascontiguousarray(np.asarray(m.get_Y()[30 + 7 * k], dtype=np.float64) + 0.01)


def _readout(pf):
    return pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), pf.log_likelihood()


def _assert_same(ref_out, ref_state, out, pf, what):
    for k, ((p1, m1, l1), (p2, m2_, l2)) in enumerate(zip(ref_out, out)):
        assert np.array_equal(p1, p2), f"{what}: posterior, frame {k}"
        assert np.array_equal(m1, m2_), f"{what}: mean, frame {k}"
        assert l1 == l2, f"{what}: likelihood, frame {k}"
    st = pf.export_state()
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(ref_state[key], st[key]), f"{what}: {key}"


def _reference(m, T, P, rng, resample, draws=None, cutoff=False):
    from gpmdm_amd import GPMDM_PF
    torch.manual_seed(5)
    pf = GPMDM_PF(m, T, P, rng=rng, seed=21 if rng == "philox" else None, resample=resample, obs_cutoff=cutoff)
    out = []
    for k in range(FRAMES):
        if draws is None:
            pf.update(_z(m, k))
        else:
            pf.update_with_draws(_z(m, k), *draws[k])
        out.append(_readout(pf))
    return out, pf.export_state()


@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("rng,resample", [("philox", "multinomial"), ("philox", "systematic"),
                                          ("torch", "multinomial")])
def test_devices_loopback_is_bitwise_one_rank(m2, R, rng, resample):
    """One process, R ranks on device 0 (gpmdm_pf_propagate_multi with loopback
    communicators): every frame bitwise the one-rank filter, uneven shards (P = 10,007)."""
    from gpmdm_amd import GPMDM_PF
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    P = 10_007
    ref_out, ref_state = _reference(m2, T, P, rng, resample)
    torch.manual_seed(5)
    pf = GPMDM_PF(m2, T, P, rng=rng, seed=21 if rng == "philox" else None, resample=resample,
                  devices=[0] * R, transport="loopback")
    out = []
    for k in range(FRAMES):
        pf.update(_z(m2, k))
        out.append(_readout(pf))
    _assert_same(ref_out, ref_state, out, pf, f"devices R={R} {rng} {resample}")


def _threaded(m, T, P, R, rng, resample, pad, draws=None, cutoff=False, splits=None):
    """R filters of shard=(R, r), each on a thread and a stream of its own, exchanging
    through loopback communicators; returns each rank's read-outs and its filter."""
    from gpmdm_amd import GPMDM_PF
    from gpmdm_amd.distributed import LoopbackComms
    comms = LoopbackComms([0] * R)
    ranks = []
    for r in range(R):
        torch.manual_seed(5)
        pf = GPMDM_PF(m, T, P, rng=rng, seed=21, resample=resample, shard=(R, r), obs_cutoff=cutoff)
        if splits:
            pf.set_obs_cutoff(True, split=splits[r % len(splits)])
        pf.set_comm(comms[r], pad_rows=pad)
        ranks.append(pf)
    outs = [[] for _ in range(R)]
    errs = []

    def run(r):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                for k in range(FRAMES):
                    if draws is None:
                        ranks[r].update(_z(m, k))
                    else:
                        ranks[r].update_with_draws(_z(m, k), *draws[k])
                    outs[r].append(_readout(ranks[r]))
                torch.cuda.current_stream().synchronize()
        except Exception as e:                  # reported on the main thread
            errs.append((r, repr(e)))

    th = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank did not finish (collective stuck)"
    assert not errs, errs
    return outs, ranks, comms


@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("P,pad", [(10_007, False), (10_008, True)])
@pytest.mark.parametrize("resample", ["multinomial", "systematic"])
def test_threaded_ranks_loopback_is_bitwise_one_rank(m2, R, P, pad, resample):
    """R ranks on R threads, each with its own stream and loopback communicator
    (gpmdm_pf_set_comm -> gpmdm_pf_propagate exchanges by itself), Philox draws: every rank's
    frames bitwise the one-rank filter."""
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    ref_out, ref_state = _reference(m2, T, P, "philox", resample)
    outs, ranks, comms = _threaded(m2, T, P, R, "philox", resample, pad)
    for r in range(R):
        _assert_same(ref_out, ref_state, outs[r], ranks[r], f"thread rank {r}/{R} P={P} pad={pad} {resample}")
    del ranks
    comms.destroy()


@pytest.mark.parametrize("R", [2, 4, 8])
def test_threaded_ranks_loopback_replay_draws(m2, R):
    """Replay draws (explicit streams, the same on every rank) through the threaded loopback
    exchange, uneven shards, multinomial: bitwise the one-rank filter."""
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    P, C, d = 10_007, 2, m2.d
    g = np.random.default_rng(17)
    draws = [(g.exponential(size=(P, C)), g.standard_normal((P, d)), g.random(P)) for _ in range(FRAMES)]
    ref_out, ref_state = _reference(m2, T, P, "torch", "multinomial", draws)
    outs, ranks, comms = _threaded(m2, T, P, R, "torch", "multinomial", False, draws)
    for r in range(R):
        _assert_same(ref_out, ref_state, outs[r], ranks[r], f"replay rank {r}/{R}")
    del ranks
    comms.destroy()


@pytest.mark.parametrize("R", [2, 4])
def test_threaded_ranks_loopback_obs_cutoff(m2, R):
    """The opt-in observation cutoff through the library's exchange: R threaded ranks with
    obs_cutoff=True, their particle tiles scheduled by different policies (whole tiles, the
    chunk grid, every tile split), bitwise the one-rank cutoff filter (the flush is per value,
    so a particle's likelihood does not depend on its tile-mates or its rank)."""
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    P = 10_007
    m2.enable_obs_cutoff(True)
    try:
        ref_out, ref_state = _reference(m2, T, P, "philox", "multinomial", cutoff=True)
        outs, ranks, comms = _threaded(m2, T, P, R, "philox", "multinomial", False, cutoff=True,
                                       splits=("auto", "chunks", "all"))
        for r in range(R):
            _assert_same(ref_out, ref_state, outs[r], ranks[r], f"cutoff rank {r}/{R}")
        del ranks
        comms.destroy()
    finally:
        m2.enable_obs_cutoff(False)


def test_loopback_validates(m2):
    """A loopback communicator of the wrong size is refused as an RCCL one is; destroying
    twice-live handles works in any order."""
    from gpmdm_amd import GPMDM_PF
    from gpmdm_amd.distributed import LoopbackComms
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    comms = LoopbackComms([0, 0, 0])
    pf = GPMDM_PF(m2, T, 1000, rng="philox", seed=1, shard=(2, 0))
    with pytest.raises(ValueError, match="size/rank"):
        pf.set_comm(comms[0])
    pf3 = GPMDM_PF(m2, T, 1000, rng="philox", seed=1, shard=(3, 1))
    with pytest.raises(ValueError, match="size/rank"):
        pf3.set_comm(comms[0])                    # rank 0's communicator for rank 1
    pf3.set_comm(comms[1])
    pf3.set_comm(None)
    comms.destroy()
    with pytest.raises(ValueError):
        GPMDM_PF(m2, T, 100, devices=[0, 0], transport="nope")
