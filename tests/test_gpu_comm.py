"""GPU: the C ABI's own exchange over an RCCL communicator (gpmdm_pf_set_comm, SURVEY.md
§8(b)'s rccl_comm).

With a communicator the library all-gathers each rank's {class, state} rows on its own
stream while the observation GP runs, then {ll}, and unpacks on the caller's stream --
the exchange point of the reference's single-process filter (gpmdm_pf.py:194-213).  RCCL
refuses two ranks on one device, so on a one-GPU box the communicator has one rank: the
exchange then moves that rank's rows through the same code (pack -> ncclAllGather on the
library stream -> events -> unpack), and GPMDM_COMM_PAD_ROWS forces the uneven-shard path
(staging buffer + copy-down).  Every variant must be bitwise the filter without one."""
import numpy as np
import pytest
import torch

from conftest import product_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from gpmdm_amd.distributed import RcclComm
    c = RcclComm.single(0)
    yield c
    c.destroy()


def _run(m, T, P, rng, comm=None, pad=False, frames=4, resample="multinomial"):
    from gpmdm_amd import GPMDM_PF
    torch.manual_seed(5)
    pf = GPMDM_PF(m, T, P, rng=rng, seed=21 if rng == "philox" else None, resample=resample)
    if comm is not None:
        pf.set_comm(comm, pad_rows=pad)
    Y = m.get_Y()
    out = []
    for k in range(frames):
        pf.update(np.asarray(Y[30 + 7 * k], dtype=np.float64) + 0.01)
        out.append((pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), pf.log_likelihood()))
    return pf, out


def _same(a, b):
    pa, oa = a
    pb, ob = b
    for (p1, m1, l1), (p2, m2, l2) in zip(oa, ob):
        assert np.array_equal(p1, p2) and np.array_equal(m1, m2) and l1 == l2
    sa, sb = pa.export_state(), pb.export_state()
    for k in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(sa[k], sb[k]), k


@pytest.mark.parametrize("rng,P", [("philox", 100_000), ("philox", 20_011), ("torch", 3001)])
def test_library_exchange_is_bitwise_the_single_rank_filter(fx_config2, comm, rng, P):
    m = product_model(fx_config2)
    T = torch.tensor(np.asarray(fx_config2["T"], dtype=np.float64))
    ref = _run(m, T, P, rng)
    _same(ref, _run(m, T, P, rng, comm))
    _same(ref, _run(m, T, P, rng, comm, pad=True))


def test_step_with_comm_and_systematic(fx_config2, comm):
    """gpmdm_pf_step accepts a communicator; systematic resampling through the exchange."""
    m = product_model(fx_config2)
    T = torch.tensor(np.asarray(fx_config2["T"], dtype=np.float64))
    _same(_run(m, T, 50_000, "philox", resample="systematic"),
          _run(m, T, 50_000, "philox", comm, pad=True, resample="systematic"))


def test_set_comm_validates(fx_config2, comm):
    from gpmdm_amd import GPMDM_PF, GPMDM_PF_Bank
    m = product_model(fx_config2)
    T = torch.tensor(np.asarray(fx_config2["T"], dtype=np.float64))
    pf = GPMDM_PF(m, T, 1000, rng="philox", seed=1, shard=(2, 0))
    with pytest.raises(ValueError, match="size/rank"):
        pf.set_comm(comm)                                  # a 1-rank comm for a 2-rank filter
    bank = GPMDM_PF_Bank(m, T, 3, 100, seed=1)
    from gpmdm_amd import _lib
    import ctypes
    rc = _lib.load().gpmdm_pf_set_comm(bank._h, ctypes.c_void_p(comm.ptr), 0)
    assert rc == _lib.GPMDM_E_INVALID
    pf1 = GPMDM_PF(m, T, 1000, rng="philox", seed=1)
    pf1.set_comm(comm)
    pf1.set_comm(None)                                     # detach: back to the plain path
    pf1.update(np.zeros(m.D))
