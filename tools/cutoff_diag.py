"""Diagnostics of the observation-GP cutoff (GPMDM_PF(obs_cutoff=True)) against the dense
kernel from the same state with the same draws: log-likelihood and weight differences, for
the model's tau and for a cutoff image whose tau is so small that nothing is flushed or
skipped (sigma2 = 1e-200: isolates the symmetric image and the epilogue from the skipping).

    python tools/cutoff_diag.py [--fixture config1_n500_p100_f200 | config2_n2000_p1000] [--P 100]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="config1_n500_p100_f200")
    ap.add_argument("--P", type=int, default=0)
    ap.add_argument("--frames", default="0,1,2,5,20")
    a = ap.parse_args()
    from conftest import load_fixture, product_model
    from gpmdm_amd import GPMDM_PF, _lib
    f = load_fixture(a.fixture)
    pre = "traj_" if "traj_E" in f else "step_"
    m = product_model(f)
    T = torch.tensor(f["T"])
    P = a.P or f[pre + "E"].shape[1]
    out = {"fixture": a.fixture, "P": P, "frames": {}}

    def run(pf, k):
        pf.load_state(f[pre + "pre_states"][k][:P], f[pre + "pre_classes"][k][:P])
        z_off = 0 if pre == "traj_" else f["z"].shape[0] - f[pre + "E"].shape[0]
        pf.update_with_draws(f["z"][k + z_off], f[pre + "E"][k][:P], f[pre + "normals"][k][:P], f[pre + "u"][k][:P])
        return pf.export_state()

    dense = GPMDM_PF(m, T, P, rng="torch")
    frames = [int(x) for x in a.frames.split(",") if int(x) < f[pre + "E"].shape[0]]
    ref = {k: run(dense, k) for k in frames}
    m.enable_obs_cutoff(True)
    out["tau"] = m.obs_cutoff_tau
    cut = GPMDM_PF(m, T, P, rng="torch", obs_cutoff=True)
    cut.set_obs_cutoff(True, stats=True)

    def cmp(name, pf):
        for k in frames:
            pf.obs_cutoff_stats(reset=True)
            st = run(pf, k)
            s = pf.obs_cutoff_stats()
            r = ref[k]
            out["frames"].setdefault(str(k), {})[name] = {
                "ll_maxabs": float(np.max(np.abs(st["ll"] - r["ll"]))),
                "w_nrel": float(np.max(np.abs(st["w"] - r["w"])) / np.max(np.abs(r["w"]))),
                "classes_equal": bool(np.array_equal(st["classes"], r["classes"])),
                "idx_equal": bool(np.array_equal(st["resample_idx"], r["resample_idx"])),
                "run_fraction": s["fraction_run"]}

    cmp("cutoff", cut)
    # a cutoff image with a vanishing tau (~1e-320): nothing flushed, no K-step skipped
    lib = _lib.load()
    Ry = None
    m._obs_cutoff = False
    m._precompute_kernel_inverses()           # a fresh image without the cutoff
    m._obs_cutoff = True
    N = m.X.shape[0]
    # rebuild through the library call with sigma2 = 1e-300
    import gpmdm_amd.model as M
    orig = M.GPMDM._install_obs_cutoff

    def tiny(self, Ry_, beta):
        with torch.no_grad():
            R = torch.as_tensor(Ry_, dtype=torch.float64)
            K_inv = np.ascontiguousarray((R @ R.T).numpy())
        beta = np.ascontiguousarray(beta, dtype=np.float64)
        y_absmax = np.ascontiguousarray(np.max(np.abs(np.asarray(self.get_Y(), dtype=np.float64)), axis=0))
        _lib.check(lib.gpmdm_model_set_obs_cutoff(self._handle, _lib.dptr(K_inv), _lib.dptr(beta),
                                                  ctypes.c_double(1e-200), _lib.dptr(y_absmax)), "tiny")
    M.GPMDM._install_obs_cutoff = tiny
    m._precompute_kernel_inverses()
    M.GPMDM._install_obs_cutoff = orig
    out["tau_tiny"] = m.obs_cutoff_tau
    cut2 = GPMDM_PF(m, T, P, rng="torch", obs_cutoff=True)
    cut2.set_obs_cutoff(True, stats=True)
    cmp("cutoff_tiny_tau", cut2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
