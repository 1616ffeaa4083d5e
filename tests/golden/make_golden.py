"""Generate the golden fixtures under tests/golden/ from the UNMODIFIED reference.

Run here only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

The reference (`/root/reference/gpmdm`) is imported read-only.  Two of its imports are
absent from this image (``torchtyping``, ``termcolor``); trivial stand-ins are written
to a temporary directory at run time (never into the repo).  The reference has no
tests or golden vectors of its own, so these fixtures are what pins the
oracle.  Each fixture holds only numbers: model inputs, random draws and the
reference's outputs.

Random draws are captured, not guessed: before each reference stage the global torch
RNG state is saved; afterwards the same shapes are re-drawn from a generator started
at that state (``gpmdm_amd.replay``) and the generator must end in exactly the state the
reference left behind.
"""
from __future__ import annotations

import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent

sys.path.insert(0, str(REPO))
from gpmdm_amd import replay, synthetic  # noqa: E402


def _import_reference():
    stub = Path(tempfile.mkdtemp(prefix="gpmdm_ref_stubs_"))
    (stub / "torchtyping").mkdir()
    (stub / "torchtyping" / "__init__.py").write_text(
        "class TensorType:\n    def __class_getitem__(cls, item):\n        return cls\n")
    (stub / "termcolor").mkdir()
    (stub / "termcolor" / "__init__.py").write_text("def cprint(*a, **k):\n    print(*a)\n")
    sys.path.insert(0, str(stub))
    sys.path.insert(0, str(REF))
    sys.dont_write_bytecode = True
    from gpmdm import GPMDM, GPMDM_PF  # noqa: WPS433
    return GPMDM, GPMDM_PF


GPMDM, GPMDM_PF = _import_reference()


def build_reference_model(C, S, L, D, d, sigma_n, seed=0):
    data = synthetic.make_sequences(C, S, L, D, d, seed=seed)
    hp = synthetic.default_hyperparameters(D, d, sigma_n)
    m = GPMDM(D=D, d=d, n_classes=C, dyn_target="full", dyn_back_step=1,
              y_lambdas_init=torch.tensor(hp["y_lambdas_init"]),
              y_lengthscales_init=torch.tensor(hp["y_lengthscales_init"]),
              y_sigma_n_init=hp["y_sigma_n_init"],
              x_lambdas_init=torch.tensor(hp["x_lambdas_init"]),
              x_lengthscales_init=torch.tensor(hp["x_lengthscales_init"]),
              x_sigma_n_init=hp["x_sigma_n_init"],
              x_lin_coeff_init=torch.tensor(hp["x_lin_coeff_init"]))
    for c in range(C):
        for Y in data.sequences[c]:
            m.add_data(Y, c)
    m.init_X()
    return m, data


def model_arrays(m):
    seq = np.array([[s.shape[0] for s in cls] for cls in m.class_aware_observations_list], dtype=np.int64)
    return dict(
        X=m.X.detach().numpy().astype(np.float64),
        Y=m.get_Y().astype(np.float64),
        seq_lengths=seq,
        y_log_lengthscales=m.y_log_lengthscales.detach().numpy(),
        y_log_lambdas=m.y_log_lambdas.detach().numpy(),
        y_log_sigma_n=np.float64(m.y_log_sigma_n.detach().item()),
        x_log_lengthscales=m.x_log_lengthscales.detach().numpy(),
        x_log_lambdas=m.x_log_lambdas.detach().numpy(),
        x_log_sigma_n=np.float64(m.x_log_sigma_n.detach().item()),
        x_log_lin_coeff=m.x_log_lin_coeff.detach().numpy(),
        sigma_n_num_X=np.float64(m.sigma_n_num_X),
        sigma_n_num_Y=np.float64(m.sigma_n_num_Y),
    )


def op_goldens(m, n_dyn, n_obs, seed):
    """Reference predictive maps at fixed query points near the training latents."""
    rng = np.random.RandomState(seed)
    X = m.X.detach().numpy()
    out = {}
    with torch.no_grad():
        for c in range(m.n_classes):
            Xc = m.get_X_for_class(c).detach().numpy()
            xs = Xc[rng.randint(0, Xc.shape[0], n_dyn)] + 0.05 * rng.randn(n_dyn, X.shape[1])
            mu, var = m.map_x_dynamics_for_class(torch.tensor(xs), class_index=c)
            out[f"dyn{c}_xs"], out[f"dyn{c}_mu"], out[f"dyn{c}_var"] = xs, mu.numpy(), var.numpy()
        xs = X[rng.randint(0, X.shape[0], n_obs)] + 0.05 * rng.randn(n_obs, X.shape[1])
        mu, var = m.map_x_to_y(torch.tensor(xs))
        out["obs_xs"], out["obs_mu"], out["obs_var"] = xs, mu.numpy(), var.numpy()
    return out


def _replay_check(state_before, draw_fn):
    g = torch.Generator()
    g.set_state(state_before)
    val = draw_fn(g)
    assert torch.equal(g.get_state(), torch.get_rng_state()), "RNG consumption mismatch"
    return val


def run_filter(m, T, P, frames, z, seed, record_from=0):
    """Drive the reference filter stage by stage and capture every draw."""
    C, d = m.n_classes, m.d
    torch.manual_seed(seed)
    st = torch.get_rng_state()
    pf = GPMDM_PF(m, markov_switching_model=torch.tensor(T), num_particles=P)
    counts = pf._divide_into_n_parts(P, C)
    sizes = [m.get_X_for_class(c).shape[0] for c in range(C)]
    init_idx = _replay_check(st, lambda g: replay.init_draws(sizes, counts, g))
    rec = {k: [] for k in ["E", "normals", "u", "pre_states", "pre_classes", "classes_switched",
                           "states_propagated", "ll", "log_w", "w", "states", "classes",
                           "posterior", "mean", "lik", "most_likely"]}
    for f in range(frames):
        pre_s = pf._particle_states.detach().numpy().copy()
        pre_c = pf._particle_classes.numpy().copy()
        zt = torch.tensor(z[f], dtype=m.dtype)
        with torch.no_grad():
            st = torch.get_rng_state()
            pf._propogate_markov_switching()
            E = _replay_check(st, lambda g: replay.switch_draws(P, C, g))
            cls1 = pf._particle_classes.numpy().copy().reshape(-1)
            cnt = [int((cls1 == c).sum()) for c in range(C)]
            st = torch.get_rng_state()
            pf._propogate_dynamics()
            nrm = _replay_check(st, lambda g: replay.dynamics_draws(cnt, d, g))
            st1 = pf._particle_states.detach().numpy().copy()
            pf._update_weights(zt)
            st = torch.get_rng_state()
            pf._resample()
            u = _replay_check(st, lambda g: replay.resample_draws(P, g))
            post = pf.class_probabilities().numpy()
            ml = pf.get_most_likely_class()
            mean = pf.current_state_mean().detach().numpy()
            lik = pf.log_likelihood()
        if f < record_from:
            continue
        rec["pre_states"].append(pre_s)
        rec["pre_classes"].append(pre_c)
        rec["E"].append(E)
        rec["normals"].append(nrm)
        rec["u"].append(u)
        rec["classes_switched"].append(cls1)
        rec["states_propagated"].append(st1)
        rec["ll"].append(pf._log_likelihoods.detach().numpy().copy())
        rec["log_w"].append(pf._log_weights.detach().numpy().copy())
        rec["w"].append(pf._weights.detach().numpy().copy())
        rec["states"].append(pf._particle_states.detach().numpy().copy())
        rec["classes"].append(pf._particle_classes.numpy().copy())
        rec["posterior"].append(post)
        rec["mean"].append(mean)
        rec["lik"].append(lik)
        rec["most_likely"].append(ml)
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["init_idx"] = np.concatenate(init_idx)
    out["init_counts"] = np.asarray(counts, dtype=np.int64)
    return out


def save(name, arrays):
    path = OUT / name
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({path.stat().st_size / 1e6:.2f} MB)")


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    # ---- config 1: N=500, D=62, d=3, C=2, P=100, 200 frames, sigma_n=0.1 -------------
    cfg = synthetic.CONFIGS[1]
    m, data = build_reference_model(cfg["C"], cfg["S"], cfg["L"], cfg["D"], cfg["d"], 0.1)
    T = synthetic.markov_matrix(cfg["C"])
    z = data.observation_stream(cfg["frames"], seed=1)
    arr = model_arrays(m)
    arr.update(op_goldens(m, 64, 128, seed=5))
    arr["T"] = T
    arr["z"] = z
    traj = run_filter(m, T, cfg["P"], cfg["frames"], z, seed=11)
    # the full per-frame particle arrays are kept for the trajectory (P=100 is small)
    arr.update({f"traj_{k}": v for k, v in traj.items()})
    save("config1_n500_p100_f200.npz", arr)

    # ---- sigma_n = 0.01 stress model, per-step (resynced) only -------------------------
    m2, data2 = build_reference_model(cfg["C"], cfg["S"], cfg["L"], cfg["D"], cfg["d"], 0.01)
    z2 = data2.observation_stream(8, seed=1)
    arr = model_arrays(m2)
    arr.update(op_goldens(m2, 32, 64, seed=6))
    arr["T"] = T
    arr["z"] = z2
    tr = run_filter(m2, T, 200, 8, z2, seed=12, record_from=5)
    arr.update({f"step_{k}": v for k, v in tr.items()})
    save("stress_n500_sigma001.npz", arr)

    # ---- config-2 model shape: N=2000, D=62, d=3, C=2; P=1000 for 3 recorded frames ----
    cfg = synthetic.CONFIGS[2]
    m3, data3 = build_reference_model(cfg["C"], cfg["S"], cfg["L"], cfg["D"], cfg["d"], 0.1)
    z3 = data3.observation_stream(5, seed=1)
    arr = model_arrays(m3)
    arr["Y"] = arr["Y"].astype(np.float32)   # f32-valued observations: store compactly
    arr.update(op_goldens(m3, 128, 256, seed=7))
    arr["T"] = T
    arr["z"] = z3
    tr = run_filter(m3, T, 1000, 5, z3, seed=13, record_from=2)
    arr.update({f"step_{k}": v for k, v in tr.items()})
    save("config2_n2000_p1000.npz", arr)


if __name__ == "__main__":
    main()
