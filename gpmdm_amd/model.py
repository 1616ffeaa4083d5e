"""GPMDM host model: the part of the reference ``GPMDM`` class the particle filter needs.

Mirrors ``/root/reference/gpmdm/gpmdm.py`` (class GPMDM, lines 18-1414) for construction,
data registry, latent initialisation, kernel-inverse precompute, persistence and the two
predictive maps; the predictive maps and everything per frame run in libgpmdm_hip.so.
Training (``gpdm_loss`` / ``train_adam``, gpmdm.py:550-885) runs
on the model's GPU in ``gpmdm_amd/training.py`` and re-uploads the device model when it
finishes; ``set_training_mode`` / ``set_evaluation_mode`` (gpmdm.py:239-279) set the
parameters' ``requires_grad`` as the reference does.  ``GPMDM`` is a ``torch.nn.Module``
with the reference's parameters (see the class docstring).

Precompute follows the reference recipe (gpmdm.py:1284-1305) on class blocks only:
``U = chol(K, upper)``, ``R = U^-1``, ``K^-1 = R R^T``.  The library keeps ``R`` (upper
triangular) and the mean weights ``beta = K_y^-1 Y`` and ``alpha_c = A_c Xout_c``; the
dense ``(C+1) x Nx x Nx`` masks of the reference are never formed.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np
import torch

from . import _lib


def _to_np(x, dtype=np.float64):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.asarray(x, dtype=dtype)


def _sq_dist(X1, X2, log_ls):
    """gpmdm.py:483-517 (expansion form), used for the setup kernel matrices."""
    ls = torch.exp(log_ls)
    a = X1 / ls
    b = X2 / ls
    return (a * a).sum(1, keepdim=True) + (b * b).sum(1, keepdim=True).T - 2.0 * (a @ b.T)


def _lin(X1, X2, log_c):
    """gpmdm.py:520-548."""
    S = torch.diag(torch.exp(log_c) ** 2)
    o1 = torch.ones(X1.shape[0], 1, dtype=X1.dtype, device=X1.device)
    o2 = torch.ones(X2.shape[0], 1, dtype=X2.dtype, device=X2.device)
    X1 = torch.cat([X1, o1], 1)
    X2 = torch.cat([X2, o2], 1)
    return X1 @ (S @ X2.T)


def _chol_inv_factor(K, what):
    """Upper Cholesky + inverse as gpmdm.py:1287-1289; returns R = U^-1 (upper)."""
    U, info = torch.linalg.cholesky_ex(K, upper=True)
    if int(info) != 0:
        # The reference ignores `info` and silently propagates garbage; we refuse.
        raise RuntimeError(f"{what}: kernel matrix is not positive definite (cholesky info={int(info)})")
    R = torch.inverse(U)
    return torch.triu(R)


def read_reference_checkpoint(path):
    """(config_dict, state_dict) of a checkpoint written by the reference's GPMDM.save
    (gpmdm.py:1307-1346): ``torch.save({'state_dict', 'config_dict'})``.  The reference's
    own loader (gpmdm.py:1368) calls ``torch.load`` with the default, which torch >= 2.6
    refuses for these files (numpy arrays in config_dict).  Here only the safe loader runs:
    ``weights_only=True`` with numpy's array reconstruction allow-listed; nothing else is
    unpickled."""
    safe = [np.ndarray, np.dtype]
    try:
        safe.append(np._core.multiarray._reconstruct)
    except AttributeError:
        safe.append(np.core.multiarray._reconstruct)
    for name in dir(np.dtypes):
        obj = getattr(np.dtypes, name)
        if isinstance(obj, type) and name.endswith("DType"):
            safe.append(obj)
    with torch.serialization.safe_globals(safe):
        save_dict = torch.load(path, weights_only=True, map_location="cpu")
    return save_dict["config_dict"], save_dict["state_dict"]


class GPMDM(torch.nn.Module):
    """Gaussian Process Multi-Dynamical Model -- inference-side mirror of gpmdm.py:GPMDM.

    A ``torch.nn.Module`` like the reference's (gpmdm.py:18): the seven log-hyperparameters
    and the latents ``X`` are ``nn.Parameter``s registered in the reference's order
    (gpmdm.py:201-230, 773), so ``state_dict`` / ``load_state_dict`` / ``parameters`` /
    ``named_parameters`` / ``train()`` / ``eval()`` / ``requires_grad`` and external
    optimisers over ``parameters()`` behave as there.  The parameters live on the host
    (``.to()`` moves them as for any module); the device model -- factors and packed tile
    images in libgpmdm_hip -- lives on ``device`` and is rebuilt whenever the parameters
    change, including in-place updates by an optimiser (detected through the parameters'
    version counters on the next use).  An edit through ``.data`` (``m.X.data.mul_(2)``)
    bypasses the version counter and is not detected: call ``refresh(force=True)`` after
    one.

    Constructor arguments are those of the reference (gpmdm.py:96-109).  ``dtype`` must be
    float64 (the reference default, required for parity: SURVEY.md §8(c)).  ``device`` is
    the GPU the device model lives on (default: the current HIP device, as torch's
    ``"cuda"`` resolves it); ``flg_train_*`` are the parameters' ``requires_grad`` flags
    (gpmdm.py:96-107; ``train_adam`` trains every parameter, as the reference's does after
    ``set_training_mode('all')``).
    """

    _PARAMS = ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
               "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff", "X")

    def __init__(self, D, d, n_classes, dyn_target, dyn_back_step,
                 y_lambdas_init, y_lengthscales_init, y_sigma_n_init,
                 x_lambdas_init, x_lengthscales_init, x_sigma_n_init, x_lin_coeff_init,
                 flg_train_y_lambdas=True, flg_train_y_lengthscales=True, flg_train_y_sigma_n=True,
                 flg_train_x_lambdas=True, flg_train_x_lengthscales=True,
                 flg_train_x_sigma_n=True, flg_train_x_lin_coeff=True,
                 sigma_n_num_Y=0., sigma_n_num_X=0.,
                 dtype=torch.float64, device=None):
        super().__init__()
        if dtype != torch.float64:
            raise NotImplementedError("gpmdm_amd computes in float64 only (reference default, gpmdm.py:109)")
        if dyn_target not in ("full", "delta") or dyn_back_step not in (1, 2):
            raise ValueError("target must be either 'full' or 'delta' \n back_step must be either 1 or 2")
        self.dtype = dtype
        dev = torch.device("cuda") if device is None else torch.device(device)
        if dev.type != "cuda":
            raise ValueError("gpmdm_amd runs on the GPU: device must be a cuda (HIP) device")
        if dev.index is None:   # "cuda": the current device (torch.cuda.set_device), as torch resolves it
            dev = torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        self.device = dev
        self.D, self.d, self.n_classes = int(D), int(d), int(n_classes)
        self.dyn_target, self.dyn_back_step = dyn_target, int(dyn_back_step)
        f64 = dict(dtype=torch.float64)

        def param(v, grad, vec=True):
            t = torch.log(torch.as_tensor(_to_np(v) if vec else float(v), **f64))
            return torch.nn.Parameter(t.reshape(-1) if vec else t, requires_grad=bool(grad))

        # registration order = the reference's (its state_dict order)
        self.y_log_lengthscales = param(y_lengthscales_init, flg_train_y_lengthscales)
        self.y_log_lambdas = param(y_lambdas_init, flg_train_y_lambdas)
        self.y_log_sigma_n = param(y_sigma_n_init, flg_train_y_sigma_n, vec=False)
        self.x_log_lengthscales = param(x_lengthscales_init, flg_train_x_lengthscales)
        self.x_log_lambdas = param(x_lambdas_init, flg_train_x_lambdas)
        self.x_log_sigma_n = param(x_sigma_n_init, flg_train_x_sigma_n, vec=False)
        self.x_log_lin_coeff = param(x_lin_coeff_init, flg_train_x_lin_coeff)
        self.register_parameter("X", None)          # set by init_X / set_latents / load
        self.sigma_n_num_Y = float(sigma_n_num_Y)
        self.sigma_n_num_X = float(sigma_n_num_X)
        self.class_aware_observations_list = [[] for _ in range(self.n_classes)]
        self._handle = None
        self._extra_devices = set()  # further GPUs holding the device model (handle_on)
        self._extra_handles = {}
        self._uploaded = None       # parameter versions the device model was built from
        # where _precompute_kernel_inverses runs: None = torch on the CPU for N <= 4096 (the
        # reference's own arithmetic), the library's device factor (gpmdm_gp_factor:
        # rocSOLVER potrf/trtri) above; or force "cpu" / "device"
        self._precompute_device = None
        # GP-tile workgroup shape (include/gpmdm_hip.h GPMDM_TILE_*: 0 default, 1 64x256,
        # 2 64x512, 3 32x512); env override for A/B runs
        self.tile_shape = int(os.environ.get("GPMDM_TILE_SHAPE", "0"))
        self._trainable = {}        # set_training_mode (gpmdm.py:247-279); empty = all
        flags = dict(y_lambdas=flg_train_y_lambdas, y_lengthscales=flg_train_y_lengthscales,
                     y_sigma_n=flg_train_y_sigma_n, x_lambdas=flg_train_x_lambdas,
                     x_lengthscales=flg_train_x_lengthscales, x_sigma_n=flg_train_x_sigma_n,
                     x_lin_coeff=flg_train_x_lin_coeff)
        self.flg_trainable_list = [k for k, v in flags.items() if v]
        self.generation = 0         # bumped by every device upload (filters rebind to it)
        self._obs_cutoff = False    # build the observation GP's cutoff image (enable_obs_cutoff)

    # ---- parameters ---------------------------------------------------------------
    def _host(self, name: str) -> torch.Tensor:
        """A detached host (CPU) view of a parameter."""
        return getattr(self, name).detach().cpu()

    def _set_param(self, name: str, value) -> None:
        """Install a parameter value: in place when the shape matches (keeps requires_grad
        and any optimiser's reference), a new Parameter otherwise."""
        t = torch.as_tensor(_to_np(value), dtype=torch.float64)
        cur = getattr(self, name, None)
        if isinstance(cur, torch.nn.Parameter) and cur.shape == t.shape:
            with torch.no_grad():
                cur.copy_(t.to(cur.device))
        else:
            grad = cur.requires_grad if isinstance(cur, torch.nn.Parameter) else True
            setattr(self, name, torch.nn.Parameter(t.clone(), requires_grad=grad))

    def _param_versions(self):
        # (this module has no submodules: its own parameter table is named_parameters())
        return tuple((n, p.data_ptr(), p._version) for n, p in self._parameters.items() if p is not None)

    def _refresh(self) -> None:
        """Rebuild the device model when the parameters changed since it was built (an
        optimiser step over parameters(), a .to(), an in-place edit)."""
        if self.X is not None and self._handle is not None and self._uploaded != self._param_versions():
            self._precompute_kernel_inverses()

    def refresh(self, force: bool = False) -> None:
        """Rebuild the device model if the parameters changed (``force``: always -- after
        edits through ``.data``, which the parameters' version counters do not see).
        Filters built on the model rebind on their next call."""
        if force and self.X is not None:
            self._precompute_kernel_inverses()
        else:
            self._refresh()

    # ---- reference API: data registry (gpmdm.py:239-309) -------------------------
    def set_evaluation_mode(self):
        """gpmdm.py:239-245: every parameter's requires_grad off."""
        self.flg_trainable_list = []
        for prm in self.parameters():
            prm.requires_grad = False

    # ---- reference API: training (gpmdm.py:247-279, 550-628, 721-885) ---------------
    _Y_PARAMS = ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n")
    _X_PARAMS = ("x_log_lengthscales", "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff")

    def set_training_mode(self, model='all'):
        """gpmdm.py:247-279: which parameters ``train_adam``'s optimiser updates."""
        if model == 'all':
            self._trainable = {n: True for n in self._Y_PARAMS + self._X_PARAMS + ("X",)}
        elif model == 'latent':
            self._trainable = {**{n: True for n in self._Y_PARAMS}, **{n: False for n in self._X_PARAMS}}
        elif model == 'dynamics':
            self._trainable = {**{n: False for n in self._Y_PARAMS}, **{n: True for n in self._X_PARAMS}}
        else:
            raise ValueError('model must be \'all\', \'latent\' or \'dynamics\'')
        for n, flag in self._trainable.items():       # X keeps its flag for 'latent' / 'dynamics'
            prm = getattr(self, n, None)
            if prm is not None:
                prm.requires_grad = flag

    def get_y_neg_log_likelihood(self, Y, X, N):
        """gpmdm.py:550-590 on the model's device (fp64 Cholesky + triangular solve); returns
        a device scalar.  ``Y``/``X`` may be host or device arrays."""
        from . import training
        f64 = dict(dtype=torch.float64, device=self.device)
        p = {n: getattr(self, n).to(**f64) for n in self._Y_PARAMS}
        p["X"] = torch.as_tensor(_to_np(X) if not isinstance(X, torch.Tensor) else X).to(**f64)
        Y = torch.as_tensor(_to_np(Y) if not isinstance(Y, torch.Tensor) else Y).to(**f64)
        return training.y_neg_log_likelihood(p, Y, self.sigma_n_num_Y)

    def get_x_neg_log_likelihood(self, Xout, Xin):
        """gpmdm.py:592-628 (class-masked K_x, evaluated block by block) on the device."""
        from . import training
        f64 = dict(dtype=torch.float64, device=self.device)
        p = {n: getattr(self, n).to(**f64) for n in self._X_PARAMS}
        Xin = torch.as_tensor(Xin).to(**f64)
        Xout = torch.as_tensor(Xout).to(**f64)
        return training.x_neg_log_likelihood(p, Xin, Xout, self._class_dynamics_rows(), self.sigma_n_num_X)

    def gpdm_loss(self, Y, N, M=None, balance=1):
        """gpmdm.py:721-760: L_y + balance * L_x (``M`` is unused, as in the reference, which
        reads its own mask)."""
        Xin, Xout, _ = self.get_Xin_Xout_matrices()
        return self.get_y_neg_log_likelihood(Y, self.X, N) + balance * self.get_x_neg_log_likelihood(Xout, Xin)

    def train_adam(self, num_opt_steps: int, num_print_steps: int = 0, lr: float = 0.01, balance: float = 1):
        """gpmdm.py:817-885 on the GPU (gpmdm_amd/training.py): Adam over every parameter,
        then the kernel-inverse precompute and device upload.  Returns the losses."""
        from . import training
        self.set_training_mode('all')
        return training.train_adam(self, num_opt_steps, num_print_steps, lr, balance)

    def add_data(self, Y, class_index: int):
        """gpmdm.py:281-298."""
        if Y.shape[1] != self.D:
            raise ValueError('Y must be a N x D matrix collecting observation data!')
        self.class_aware_observations_list[class_index].append(Y)

    @property
    def observations_list(self):
        return [seq for cls in self.class_aware_observations_list for seq in cls]

    def get_Y(self) -> np.ndarray:
        """gpmdm.py:779-793 (meanY = 0)."""
        self.meanY = 0
        return np.concatenate([_to_np(y) if isinstance(y, torch.Tensor) else np.asarray(y)
                               for y in self.observations_list], 0) - self.meanY

    def get_Y_for_class(self, class_index: int) -> np.ndarray:
        """gpmdm.py:795-815."""
        self.meanY = 0
        return np.concatenate(self.class_aware_observations_list[class_index], 0) - self.meanY

    def get_X_for_class(self, class_index: int) -> torch.Tensor:
        """gpmdm.py:906-921."""
        per = [sum(len(s) for s in self.class_aware_observations_list[i]) for i in range(self.n_classes)]
        start = sum(per[:class_index])
        return self.X[start:start + per[class_index], :]

    def get_latent_sequences(self):
        """gpmdm.py:887-904."""
        X = self._host("X").numpy()
        out, s = [], 0
        for seq in self.observations_list:
            out.append(X[s:s + len(seq)])
            s += len(seq)
        return out

    def get_Xin_Xout_matrices(self, X=None, target=None, back_step=None):
        """gpmdm.py:630-718 -- all four (target, back_step) modes."""
        X = self.X if X is None else torch.as_tensor(X, dtype=torch.float64)
        target = self.dyn_target if target is None else target
        back_step = self.dyn_back_step if back_step is None else back_step
        Xin, Xout, starts, s = [], [], [], 0
        for seq in self.observations_list:
            L = len(seq)
            Xs = X[s:s + L]
            starts.append(s)
            s += L
            if back_step == 1:
                xi, xo = Xs[:-1], Xs[1:]
                if target == "delta":
                    xo = Xs[1:] - Xs[:-1]
            elif back_step == 2:
                xi = torch.cat((Xs[1:-1], Xs[:-2]), 1)
                xo = Xs[2:] if target == "full" else Xs[2:] - Xs[1:-1]
            else:
                raise ValueError("target must be either 'full' or 'delta' \n back_step must be either 1 or 2")
            if target not in ("full", "delta"):
                raise ValueError("target must be either 'full' or 'delta' \n back_step must be either 1 or 2")
            Xin.append(xi)
            Xout.append(xo)
        return torch.cat(Xin, 0), torch.cat(Xout, 0), starts

    # ---- latent init + precompute (gpmdm.py:762-777, 1275-1305) ------------------
    def init_X(self):
        """PCA initialisation of the latents (gpmdm.py:762-777), then the precompute."""
        from sklearn.decomposition import PCA   # the reference's own dependency (gpmdm.py:12)
        X0 = PCA(n_components=self.d).fit_transform(self.get_Y())
        self._set_param("X", X0)
        self._precompute_kernel_inverses()

    def set_latents(self, X):
        """Install trained latents (e.g. from a saved model) and rebuild the device model."""
        self._set_param("X", X)
        self._precompute_kernel_inverses()

    def _class_dynamics_rows(self):
        """Number of dynamics pairs per class (rows of the class-c block of Xin)."""
        lag = self.dyn_back_step
        return [sum(len(s) - lag for s in cls) for cls in self.class_aware_observations_list]

    def _precompute_kernel_inverses(self):
        if self.dyn_back_step != 1:
            raise NotImplementedError("the particle-filter path supports dyn_back_step=1 (as the "
                                      "reference PF does, gpmdm_pf.py:164)")
        N = self.X.shape[0]
        where = self._precompute_device or ("cpu" if N <= 4096 else "device")
        versions = self._param_versions()
        if where == "device":
            self._precompute_on_device()
            self._uploaded = versions
            return
        dev = torch.device("cpu")
        f64 = dict(dtype=torch.float64, device=dev)
        X = self._host("X").to(**f64)
        Y = torch.as_tensor(self.get_Y(), **f64)
        eye = lambda n: torch.eye(n, **f64)  # noqa: E731
        ylog_ls, xlog_ls = self._host("y_log_lengthscales"), self._host("x_log_lengthscales")
        xlog_c = self._host("x_log_lin_coeff")
        with torch.no_grad():
            Ky = torch.exp(-_sq_dist(X, X, ylog_ls)) + torch.exp(self._host("y_log_sigma_n")) ** 2 * eye(N) \
                + self.sigma_n_num_Y ** 2 * eye(N)
            Ry = _chol_inv_factor(Ky, "K_y")
            del Ky
            beta = (Ry @ Ry.T) @ Y
            Xin, Xout, _ = self.get_Xin_Xout_matrices(X=X.cpu())
            Xin, Xout = Xin.to(dev), Xout.to(dev)
            rows = self._class_dynamics_rows()
            off = 0
            dyn = []
            for c in range(self.n_classes):
                n_c = rows[c]
                if n_c <= 0:
                    raise ValueError(f"class {c} has no dynamics pairs")
                xi, xo = Xin[off:off + n_c], Xout[off:off + n_c]
                off += n_c
                K = torch.exp(-_sq_dist(xi, xi, xlog_ls)) + torch.exp(self._host("x_log_sigma_n")) ** 2 * eye(n_c) \
                    + self.sigma_n_num_X ** 2 * eye(n_c)
                K = K + _lin(xi, xi, xlog_c)
                K = K + 1e-6 * eye(n_c)
                Rc = _chol_inv_factor(K, f"K_x class {c}")
                alpha = (Rc @ Rc.T) @ xo
                dyn.append((xi.cpu().numpy().copy(), Rc.cpu().numpy().copy(), alpha.cpu().numpy().copy()))
            obs = (Ry.cpu().numpy().copy(), beta.cpu().numpy().copy())
        self._upload(obs, dyn)
        self._uploaded = versions

    def _precompute_on_device(self):
        """The same factors through gpmdm_gp_factor (device Gram matrix, rocSOLVER potrf +
        trtri, rocBLAS trmm), one GP block at a time."""
        lib = _lib.load()
        dev_index = self.device.index

        def factor(X, log_ls, lin_c2, a, b, c, B, what):
            X = np.ascontiguousarray(X, dtype=np.float64)
            B = np.ascontiguousarray(B, dtype=np.float64)
            n, d = X.shape
            ls = np.ascontiguousarray(_to_np(torch.exp(log_ls)))   # the descriptor's lengthscales, bit for bit
            c2 = None if lin_c2 is None else np.ascontiguousarray(lin_c2, dtype=np.float64)
            R = np.empty((n, n))
            M = np.empty((n, B.shape[1]))
            _lib.check(lib.gpmdm_gp_factor(dev_index, _lib.dptr(X), n, d, _lib.dptr(ls), _lib.dptr(c2),
                                           a, b, c, _lib.dptr(B), B.shape[1], _lib.dptr(R), _lib.dptr(M)), what)
            return R, M

        X = self._host("X").numpy()
        Y = np.asarray(self.get_Y(), dtype=np.float64)
        sy2 = float(torch.exp(self._host("y_log_sigma_n"))) ** 2
        sx2 = float(torch.exp(self._host("x_log_sigma_n"))) ** 2
        Ry, beta = factor(X, self._host("y_log_lengthscales"), None, sy2, self.sigma_n_num_Y ** 2, 0.0, Y, "K_y")
        Xin, Xout, _ = self.get_Xin_Xout_matrices(X=self._host("X"))
        Xin, Xout = _to_np(Xin), _to_np(Xout)
        c2 = _to_np(torch.exp(self._host("x_log_lin_coeff")) ** 2)
        dyn, off = [], 0
        for c, n_c in enumerate(self._class_dynamics_rows()):
            if n_c <= 0:
                raise ValueError(f"class {c} has no dynamics pairs")
            xi, xo = Xin[off:off + n_c], Xout[off:off + n_c]
            off += n_c
            Rc, alpha = factor(xi, self._host("x_log_lengthscales"), c2, sx2, self.sigma_n_num_X ** 2, 1e-6, xo,
                               f"K_x class {c}")
            dyn.append((np.ascontiguousarray(xi), Rc, alpha))
        self._upload((Ry, beta), dyn)

    def _upload(self, obs, dyn):
        lib = _lib.load()
        C, d, D = self.n_classes, self.d, self.D
        keep = []   # keep arrays alive during the call

        def arr(a):
            a = np.ascontiguousarray(a, dtype=np.float64)
            keep.append(a)
            return _lib.dptr(a)

        Ry, beta = obs
        desc = _lib.ModelDesc()
        desc.N, desc.D, desc.d, desc.C = self.X.shape[0], D, d, C
        desc.tile_shape = self.tile_shape
        desc.X = arr(self._host("X").numpy())
        desc.obs_R = arr(Ry)
        desc.obs_beta = arr(beta)
        desc.y_lengthscales = arr(torch.exp(self._host("y_log_lengthscales")).numpy())
        desc.y_inv_lambda2 = arr((torch.exp(self._host("y_log_lambdas")) ** -2).numpy())
        nc = np.asarray([x[0].shape[0] for x in dyn], dtype=np.int64)
        keep.append(nc)
        desc.Nc = _lib.i64ptr(nc)
        PtrArr = _lib._dp * C
        xin_p = PtrArr(*[arr(x[0]) for x in dyn])
        r_p = PtrArr(*[arr(x[1]) for x in dyn])
        a_p = PtrArr(*[arr(x[2]) for x in dyn])
        keep += [xin_p, r_p, a_p]
        desc.Xin, desc.dyn_R, desc.dyn_alpha = xin_p, r_p, a_p
        desc.x_lengthscales = arr(torch.exp(self._host("x_log_lengthscales")).numpy())
        desc.x_lin_coeff2 = arr((torch.exp(self._host("x_log_lin_coeff")) ** 2).numpy())
        desc.x_inv_lambda2 = arr((torch.exp(self._host("x_log_lambdas")) ** -2).numpy())
        handle = ctypes.c_void_p()
        self._release()
        _lib.check(lib.gpmdm_model_create(ctypes.byref(desc), self.device.index, ctypes.byref(handle)),
                   "gpmdm_model_create")
        self._handle = handle
        self.generation += 1
        # the same image on the other devices a multi-device filter asked for (handle_on)
        for dev in sorted(self._extra_devices):
            h = ctypes.c_void_p()
            _lib.check(lib.gpmdm_model_create(ctypes.byref(desc), int(dev), ctypes.byref(h)), "gpmdm_model_create")
            self._extra_handles[dev] = h
        if self._obs_cutoff:
            self._install_obs_cutoff()

    def _install_obs_cutoff(self):
        """The observation GP's cutoff image on every device image, built on the device from
        the model's own factor (gpmdm_model_build_obs_cutoff: R and K_y^-1 Y read back out of
        the device image, K_y^-1 = U^-1 U^-T (gpmdm.py:1286-1290) by rocBLAS dsyrk, the
        tile-major packing by a device kernel; no N x N matrix on the host)."""
        lib = _lib.load()
        y_absmax = np.ascontiguousarray(np.max(np.abs(np.asarray(self.get_Y(), dtype=np.float64)), axis=0))
        sigma2 = float(torch.exp(self._host("y_log_sigma_n"))) ** 2 + self.sigma_n_num_Y ** 2
        for h in [self._handle] + [self._extra_handles[d] for d in sorted(self._extra_handles)]:
            _lib.check(lib.gpmdm_model_build_obs_cutoff(h, ctypes.c_double(sigma2), _lib.dptr(y_absmax), None, None),
                       "gpmdm_model_build_obs_cutoff")

    def enable_obs_cutoff(self, on: bool = True):
        """Build (or drop) the observation GP's kernel-value cutoff image, which filters use
        with ``GPMDM_PF(..., obs_cutoff=True)`` (DESIGN.md §3 "Kernel-value cutoff": kernel
        values below a provable tau flushed to 0 and the MFMAs of unreachable training rows
        skipped; results equal the dense filter's to rounding).  The image is built on the
        device from the model's own factor (_install_obs_cutoff), and rebuilt with the model."""
        on = bool(on)
        if on == self._obs_cutoff:
            return
        self._obs_cutoff = on
        if self._handle is None:
            return                                  # built with the model
        if on:
            gen = self.generation
            self._refresh()                         # (a rebuilt model installs the image itself)
            if self.generation == gen:
                self._install_obs_cutoff()
        else:
            lib = _lib.load()
            for h in [self._handle] + list(self._extra_handles.values()):
                _lib.check(lib.gpmdm_model_set_obs_cutoff(h, None, None, ctypes.c_double(0.0), None),
                           "gpmdm_model_set_obs_cutoff")

    @property
    def obs_cutoff_tau(self) -> float:
        """The cutoff tau of the model's cutoff image (0.0: none)."""
        t = ctypes.c_double()
        _lib.check(_lib.load().gpmdm_model_obs_cutoff(self.handle, ctypes.byref(t)), "gpmdm_model_obs_cutoff")
        return t.value

    def handle_on(self, device_index: int):
        """The device model on GPU ``device_index`` (GPMDM_PF(devices=[...]): one image per
        device, all built from the same host factors).  The first request for a device other
        than ``self.device`` re-uploads the model to every requested device (filters rebind)."""
        dev = int(device_index)
        if dev == self.device.index:
            return self.handle
        h = self.handle and self._extra_handles.get(dev)
        if h is None:
            self._extra_devices.add(dev)
            try:
                self._precompute_kernel_inverses()
            except Exception:
                self._extra_devices.discard(dev)
                raise
            h = self._extra_handles[dev]
        return h

    def _release(self):
        if getattr(self, "_handle", None) is not None and self._handle.value:
            _lib.load().gpmdm_model_destroy(self._handle)
        self._handle = None
        for h in getattr(self, "_extra_handles", {}).values():
            if h is not None and h.value:
                _lib.load().gpmdm_model_destroy(h)
        self._extra_handles = {}

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    @property
    def handle(self):
        if self._handle is None:
            raise RuntimeError("model not initialised: call init_X() (or load a saved model)")
        self._refresh()
        return self._handle

    # ---- predictive maps (gpmdm.py:923-963, 1032-1068) --------------------------
    def _predict(self, Xstar, class_index=None):
        xs = torch.as_tensor(Xstar, dtype=torch.float64)
        out_dev = xs.device
        xs = xs.to(self.device).contiguous()
        n = xs.shape[0]
        width = self.D if class_index is None else self.d
        mu = torch.empty((n, width), dtype=torch.float64, device=self.device)
        var = torch.empty((n, width), dtype=torch.float64, device=self.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        lib = _lib.load()
        if class_index is None:
            _lib.check(lib.gpmdm_predict_obs(self.handle, xs.data_ptr(), n, mu.data_ptr(), var.data_ptr(), stream),
                       "map_x_to_y")
        else:
            _lib.check(lib.gpmdm_predict_dyn(self.handle, int(class_index), xs.data_ptr(), n,
                                             mu.data_ptr(), var.data_ptr(), stream),
                       "map_x_dynamics_for_class")
        return mu.to(out_dev), var.to(out_dev)

    def map_x_to_y(self, Xstar, flg_noise: bool = False):
        """gpmdm.py:923-963: mean and diagonal variance of the observation GP at Xstar."""
        mu, var = self._predict(Xstar)
        if flg_noise:   # gpmdm.py:988-989
            extra = float(torch.exp(self._host("y_log_sigma_n")) ** 2) + self.sigma_n_num_Y ** 2
            var = var + extra * (torch.exp(self._host("y_log_lambdas")) ** -2).to(var.device)[None, :]
        return mu, var

    def map_x_dynamics_for_class(self, Xstar, class_index: int, flg_noise: bool = False):
        """gpmdm.py:1032-1068: mean and diagonal variance of class c's dynamics GP."""
        if not 0 <= int(class_index) < self.n_classes:
            raise ValueError("class_index out of range")
        mu, var = self._predict(Xstar, class_index)
        if flg_noise:   # gpmdm.py:1095-1098
            extra = float(torch.exp(self._host("x_log_sigma_n")) ** 2) + self.sigma_n_num_X ** 2
            var = var + extra * (torch.exp(self._host("x_log_lambdas")) ** -2).to(var.device)[None, :]
        return mu, var

    # ---- kernel helpers (gpmdm.py:311-378, 381-548, 965-991, 1070-1101) ------------
    # torch fp64 on the inputs' device; the per-frame path never calls them (the tile kernel
    # generates its kernel rows itself), they serve analyses and the all-class map below.
    def _par(self, t, like):
        return t.to(device=like.device, dtype=torch.float64)

    def get_weighted_distances(self, X1, X2, log_lengthscales_par):
        """gpmdm.py:483-517 (expansion form)."""
        return _sq_dist(X1, X2, self._par(log_lengthscales_par, X1))

    def get_rbf_kernel(self, X1, X2, log_lengthscales_par, log_sigma_n_par, sigma_n_num=0, flg_noise=True):
        """gpmdm.py:436-481 (noise on the diagonal of X1's rows when flg_noise)."""
        K = torch.exp(-self.get_weighted_distances(X1, X2, log_lengthscales_par))
        if flg_noise:
            N = X1.shape[0]
            eye = torch.eye(N, dtype=torch.float64, device=X1.device)
            K = K + torch.exp(self._par(log_sigma_n_par, X1)) ** 2 * eye + sigma_n_num ** 2 * eye
        return K

    def get_lin_kernel(self, X1, X2, log_lin_coeff_par):
        """gpmdm.py:520-548."""
        return _lin(X1, X2, self._par(log_lin_coeff_par, X1))

    def get_y_kernel(self, X1, X2, flg_noise=True):
        """gpmdm.py:381-406."""
        return self.get_rbf_kernel(X1, X2, self.y_log_lengthscales, self.y_log_sigma_n, self.sigma_n_num_Y, flg_noise)

    def get_x_kernel(self, X1, X2, flg_noise=True):
        """gpmdm.py:408-434 (RBF + linear)."""
        return (self.get_rbf_kernel(X1, X2, self.x_log_lengthscales, self.x_log_sigma_n, self.sigma_n_num_X, flg_noise)
                + self.get_lin_kernel(X1, X2, self.x_log_lin_coeff))

    def get_y_diag_kernel(self, X, flg_noise=False):
        """gpmdm.py:965-991."""
        n = X.shape[0]
        k = torch.ones(n, dtype=torch.float64, device=X.device)
        if flg_noise:
            k = k + torch.exp(self._par(self.y_log_sigma_n, X)) ** 2 + self.sigma_n_num_Y ** 2
        return k

    def get_x_diag_kernel(self, X, flg_noise=False):
        """gpmdm.py:1070-1101: 1 + x~^T C^2 x~ (+ noise)."""
        c2 = torch.exp(self._par(self.x_log_lin_coeff, X)) ** 2
        k = 1.0 + (X * X) @ c2[:-1] + c2[-1]
        if flg_noise:
            k = k + torch.exp(self._par(self.x_log_sigma_n, X)) ** 2 + self.sigma_n_num_X ** 2
        return k

    def _class_rows(self):
        return [sum(len(s) - 1 for s in seqs) for seqs in self.class_aware_observations_list]

    def get_M(self):
        """gpmdm.py:311-340: block-diagonal ones, one Nx x Nx block per class (dense, as the
        reference builds it; the library itself only ever stores the class blocks)."""
        rows = self._class_rows()
        return torch.block_diag(*[torch.ones(n, n, dtype=torch.float64) for n in rows])

    def get_M_for_class(self, class_index: int):
        """gpmdm.py:342-378: the class's block of get_M, zeros elsewhere."""
        rows = self._class_rows()
        o = sum(rows[:class_index])
        M = torch.zeros(sum(rows), sum(rows), dtype=torch.float64)
        M[o:o + rows[class_index], o:o + rows[class_index]] = 1.0
        return M

    def map_x_dynamics(self, Xstar, flg_noise: bool = False):
        """gpmdm.py:993-1030: the all-class dynamics map with Kx_inv = inverse of the
        M-masked kernel (block diagonal: per class block, no 1e-6 jitter, gpmdm.py:1291-1295)
        against the unmasked K(Xin, X*), i.e. sum over classes of the class-block terms.
        Torch fp64 on the model's device, class blocks only (not on the per-frame path)."""
        if self.dyn_back_step != 1:
            raise NotImplementedError("dyn_back_step=2 models are not supported (as in the reference filter)")
        with torch.no_grad():       # a read-out, like the library's maps (no autograd graph)
            return self._map_x_dynamics(Xstar, flg_noise)

    def _map_x_dynamics(self, Xstar, flg_noise):
        dev = self.device
        xs = torch.as_tensor(Xstar, dtype=torch.float64)
        out_dev = xs.device
        xs = xs.to(dev)
        Xin, Xout, _ = self.get_Xin_Xout_matrices()
        Xin, Xout = Xin.to(dev), Xout.to(dev)
        mean = torch.zeros(xs.shape[0], self.d, dtype=torch.float64, device=dev)
        quad = torch.zeros(xs.shape[0], dtype=torch.float64, device=dev)
        o = 0
        for n in self._class_rows():
            xi, xo = Xin[o:o + n], Xout[o:o + n]
            U, _ = torch.linalg.cholesky_ex(self.get_x_kernel(xi, xi), upper=True)   # info ignored, as the reference
            Ui = torch.inverse(U)
            A = Ui @ Ui.T
            ks = self.get_x_kernel(xi, xs, False)
            mean = mean + (xo.T @ A @ ks).T
            quad = quad + torch.sum((ks.T @ A) * ks.T, dim=1)
            o += n
        vc = self.get_x_diag_kernel(xs, flg_noise) - quad
        lam = torch.exp(self._host("x_log_lambdas").to(dev)) ** -2
        return mean.to(out_dev), (vc[:, None] * lam[None, :]).to(out_dev)

    # ---- map read-outs used by train_gpmdm.ipynb (gpmdm.py:1103-1273) -------------
    def get_next_x(self, gp_mean_out, gp_out_var, Xold, flg_sample: bool = False):
        """gpmdm.py:1103-1145: the next latent state from a dynamics-GP output (the mean, or
        a draw from N(mean, var) with torch's generator; 'delta' targets add Xold)."""
        step = torch.distributions.Normal(gp_mean_out, torch.sqrt(gp_out_var)).rsample() if flg_sample else gp_mean_out
        if self.dyn_target == "full":
            return step
        if self.dyn_target == "delta":
            return Xold + step

    @staticmethod
    def _nmse(target, mu, var) -> float:
        # the reference's expression, floor division included (gpmdm.py:1192, 1235, 1269)
        return float(np.mean((target - mu) ** 2 // var))

    def get_dynamics_map_performance_for_class(self, class_index: int, flg_noise: bool = False):
        """gpmdm.py:1147-1196: class c's dynamics GP on every Xin row (all classes' rows,
        as the reference does) -> (mean, var, Xout, Xin, NMSE) as numpy arrays."""
        with torch.no_grad():
            Xin, Xout, _ = self.get_Xin_Xout_matrices(X=self._host("X"))
            mu, var = self.map_x_dynamics_for_class(Xin, class_index, flg_noise=flg_noise)
            mu, var, Xout, Xin = _to_np(mu), _to_np(var), _to_np(Xout), _to_np(Xin)
        return mu, var, Xout, Xin, self._nmse(Xout, mu, var)

    def get_latent_map_performance(self, flg_noise: bool = False):
        """gpmdm.py:1199-1239: the observation GP at the training latents ->
        (mean, var, Y, NMSE) as numpy arrays."""
        with torch.no_grad():
            mu, var = self.map_x_to_y(self._host("X"), flg_noise=flg_noise)
            mu, var = _to_np(mu), _to_np(var)
            Y = self.get_Y() + self.meanY
        return mu, var, Y, self._nmse(Y, mu, var)

    def get_latent_map_performance_for_class(self, class_index: int, flg_noise: bool = False):
        """gpmdm.py:1241-1273: as get_latent_map_performance on class c's latents."""
        with torch.no_grad():
            mu, var = self.map_x_to_y(self.get_X_for_class(class_index).detach(), flg_noise=flg_noise)
            mu, var = _to_np(mu), _to_np(var)
            Y = self.get_Y_for_class(class_index) + self.meanY
        return mu, var, Y, self._nmse(Y, mu, var)

    # ---- persistence (gpmdm.py:1307-1414) ---------------------------------------
    def config_dict(self):
        return {
            "D": self.D, "d": self.d, "n_classes": self.n_classes,
            "dyn_target": self.dyn_target, "dyn_back_step": self.dyn_back_step,
            "sigma_n_num_X": self.sigma_n_num_X, "sigma_n_num_Y": self.sigma_n_num_Y,
            "y_lengthscales_init": torch.exp(self._host("y_log_lengthscales")).tolist(),
            "y_lambdas_init": torch.exp(self._host("y_log_lambdas")).tolist(),
            "y_sigma_n_init": float(torch.exp(self._host("y_log_sigma_n"))),
            "x_lengthscales_init": torch.exp(self._host("x_log_lengthscales")).tolist(),
            "x_lambdas_init": torch.exp(self._host("x_log_lambdas")).tolist(),
            "x_sigma_n_init": float(torch.exp(self._host("x_log_sigma_n"))),
            "x_lin_coeff_init": torch.exp(self._host("x_log_lin_coeff")).tolist(),
        }

    # ---- torch.nn.Module parameter access: state_dict / parameters / named_parameters come
    # from nn.Module (registration order = the reference's, gpmdm.py:201-230, 773) -----------
    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """nn.Module.load_state_dict by the reference's names (gpmdm.py:1402), then the device
        model is rebuilt (filters built on this model rebind on their next call).  A model
        without latents yet takes X's shape from the state dict.  As nn.Module, the whole
        dict is checked before anything is installed: with ``strict`` missing / unexpected
        keys raise, and a value whose shape differs from its parameter's (X: another number
        of latents than the model holds) raises a size-mismatch error naming the key; a
        rejected dict leaves the model unchanged."""
        missing = [k for k in self._PARAMS if k not in state_dict]
        unexpected = [k for k in state_dict if k not in self._PARAMS]
        if strict and (missing or unexpected):
            raise RuntimeError(f"load_state_dict: missing keys {missing}, unexpected keys {unexpected}")
        vals = {}
        for k in self._PARAMS:
            if k not in state_dict:
                continue
            v = torch.as_tensor(_to_np(state_dict[k]))
            cur = getattr(self, k)
            if cur is None:                          # X of a model without latents yet
                if v.dim() != 2 or v.shape[1] != self.d:
                    raise RuntimeError(f"load_state_dict: size mismatch for {k}: expected (N, {self.d}), "
                                       f"got {tuple(v.shape)}")
            elif v.numel() != cur.numel() or (v.dim() > 1 and tuple(v.shape) != tuple(cur.shape)):
                raise RuntimeError(f"load_state_dict: size mismatch for {k}: copying a param with shape "
                                   f"{tuple(v.shape)}, the shape in the current model is {tuple(cur.shape)}")
            else:
                v = v.reshape(cur.shape)
            vals[k] = v
        for k, v in vals.items():
            self._set_param(k, v)
        if self.X is not None:
            self._precompute_kernel_inverses()
        return torch.nn.modules.module._IncompatibleKeys(missing, unexpected)

    def save(self, file_path) -> None:
        """gpmdm.py:1307-1346.  Writes exactly ``file_path``:

        * any suffix but ``.npz``: the reference's own layout, ``torch.save({'state_dict':
          <the 8 parameters in registration order>, 'config_dict': <the reference's 17 keys,
          observations as the arrays add_data received>})`` -- a file the reference's
          ``GPMDM.load`` and this class's ``load`` both read;
        * ``.npz``: a pickle-free archive (the torch layout holds numpy arrays, which
          ``torch.load(weights_only=True)`` reads only with numpy allow-listed)."""
        suffix = Path(file_path).suffix
        if suffix != ".npz":
            if suffix not in (".pth", ".pt"):
                import warnings
                warnings.warn(f"GPMDM.save({str(file_path)!r}): writing the reference's torch layout (a pickle) "
                              "to exactly this path; use a '.npz' suffix for the pickle-free archive",
                              stacklevel=2)
            return self._save_reference_layout(file_path)
        return self._save_npz(file_path)

    def _reference_config_dict(self):
        """The reference's config_dict (gpmdm.py:1317-1336), keys in its order."""
        def ex(t):
            return t.detach().exp()
        return {
            "class_aware_observations_list": [list(c) for c in self.class_aware_observations_list],
            "dyn_target": self.dyn_target,
            "dyn_back_step": self.dyn_back_step,
            "D": self.D, "d": self.d, "n_classes": self.n_classes,
            "sigma_n_num_X": self.sigma_n_num_X, "sigma_n_num_Y": self.sigma_n_num_Y,
            "dtype": str(self.dtype),
            "device": str(self.device),
            "y_lengthscales_init": ex(self.y_log_lengthscales).tolist(),
            "y_lambdas_init": ex(self.y_log_lambdas).tolist(),
            "y_sigma_n_init": ex(self.y_log_sigma_n).item(),
            "x_lengthscales_init": ex(self.x_log_lengthscales).tolist(),
            "x_lambdas_init": ex(self.x_log_lambdas).tolist(),
            "x_sigma_n_init": ex(self.x_log_sigma_n).item(),
            "x_lin_coeff_init": ex(self.x_log_lin_coeff).tolist(),
        }

    def _save_reference_layout(self, file_path):
        sd = self.state_dict()                 # nn.Module's: detached tensors + _metadata
        with open(file_path, "wb") as fh:     # a file object: torch.save adds no suffix
            torch.save({"state_dict": sd, "config_dict": self._reference_config_dict()}, fh)

    def _save_npz(self, file_path):
        arrays = {"X": self._host("X").numpy()}
        seq_len = []
        for c, cls in enumerate(self.class_aware_observations_list):
            for k, y in enumerate(cls):
                arrays[f"obs_{c}_{k}"] = _to_np(y, np.float64 if np.asarray(y).dtype == np.float64 else np.float32)
            seq_len.append(len(cls))
        arrays["n_seq"] = np.asarray(seq_len, dtype=np.int64)
        for k in ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
                  "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff"):
            arrays[k] = self._host(k).numpy()
        cfg = self.config_dict()
        arrays["cfg_int"] = np.asarray([cfg["D"], cfg["d"], cfg["n_classes"], cfg["dyn_back_step"]], dtype=np.int64)
        arrays["cfg_target"] = np.asarray([0 if cfg["dyn_target"] == "full" else 1], dtype=np.int64)
        arrays["cfg_num"] = np.asarray([cfg["sigma_n_num_X"], cfg["sigma_n_num_Y"]], dtype=np.float64)
        with open(file_path, "wb") as fh:     # a file object: np.savez adds no suffix
            np.savez(fh, **arrays)

    @staticmethod
    def _is_npz(path) -> bool:
        """True for a numpy archive (a zip of ``.npy`` members), False for a torch archive
        (a zip holding ``<name>/data.pkl``) or torch's legacy non-zip pickle stream; the
        file's content decides, not its suffix."""
        import zipfile
        if not zipfile.is_zipfile(path):
            return False
        with zipfile.ZipFile(path) as z:
            names = z.namelist()
        return bool(names) and all(n.endswith(".npy") for n in names)

    @classmethod
    def load(cls, file_path, flg_print: bool = False, device=None, upload: bool = True) -> "GPMDM":
        """gpmdm.py:1349-1414.  Reads either format ``save`` writes -- the reference's torch
        layout (also any file the reference itself wrote) through ``torch.load(weights_only
        =True)`` with numpy arrays allow-listed, or the pickle-free ``.npz`` -- chosen by the
        file's content.  ``upload=False`` stops before the device precompute."""
        path = Path(file_path)
        names = ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
                 "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff")
        if cls._is_npz(path):
            f = np.load(path, allow_pickle=False)
            D, d, C, bs = (int(v) for v in f["cfg_int"])
            target = "full" if int(f["cfg_target"][0]) == 0 else "delta"
            m = cls(D=D, d=d, n_classes=C, dyn_target=target, dyn_back_step=bs,
                    y_lambdas_init=np.exp(f["y_log_lambdas"]), y_lengthscales_init=np.exp(f["y_log_lengthscales"]),
                    y_sigma_n_init=float(np.exp(f["y_log_sigma_n"])), x_lambdas_init=np.exp(f["x_log_lambdas"]),
                    x_lengthscales_init=np.exp(f["x_log_lengthscales"]),
                    x_sigma_n_init=float(np.exp(f["x_log_sigma_n"])),
                    x_lin_coeff_init=np.exp(f["x_log_lin_coeff"]),
                    sigma_n_num_X=float(f["cfg_num"][0]), sigma_n_num_Y=float(f["cfg_num"][1]), device=device)
            for k in names:   # exact log-parameters (exp/log round trips can move an ulp)
                m._set_param(k, np.asarray(f[k], dtype=np.float64))
            for c in range(C):
                for k in range(int(f["n_seq"][c])):
                    m.add_data(f[f"obs_{c}_{k}"], c)
            X = f["X"]
        else:
            cfg, sd = read_reference_checkpoint(path)
            m = cls(D=cfg["D"], d=cfg["d"], n_classes=cfg["n_classes"], dyn_target=cfg["dyn_target"],
                    dyn_back_step=cfg["dyn_back_step"], y_lambdas_init=cfg["y_lambdas_init"],
                    y_lengthscales_init=cfg["y_lengthscales_init"], y_sigma_n_init=cfg["y_sigma_n_init"],
                    x_lambdas_init=cfg["x_lambdas_init"], x_lengthscales_init=cfg["x_lengthscales_init"],
                    x_sigma_n_init=cfg["x_sigma_n_init"], x_lin_coeff_init=cfg["x_lin_coeff_init"],
                    sigma_n_num_X=cfg["sigma_n_num_X"], sigma_n_num_Y=cfg["sigma_n_num_Y"], device=device)
            m.class_aware_observations_list = [list(c) for c in cfg["class_aware_observations_list"]]
            for k in names:
                m._set_param(k, sd[k].to(torch.float64))
            X = sd["X"]
        if flg_print:
            for k in names:
                print(k, "\t", getattr(m, k))
        if upload:
            m.set_latents(X)
        else:
            m._set_param("X", X)
        return m

    @classmethod
    def from_arrays(cls, X, Y_sequences, y_log_lengthscales, y_log_lambdas, y_log_sigma_n,
                    x_log_lengthscales, x_log_lambdas, x_log_sigma_n, x_log_lin_coeff,
                    sigma_n_num_X=0.0, sigma_n_num_Y=0.0, dyn_target="full", device=None):
        """Build from explicit latents / observations (Y_sequences[c] = list of arrays)."""
        D = np.asarray(Y_sequences[0][0]).shape[1]
        d = np.asarray(X).shape[1]
        m = cls(D=D, d=d, n_classes=len(Y_sequences), dyn_target=dyn_target, dyn_back_step=1,
                y_lambdas_init=np.exp(y_log_lambdas), y_lengthscales_init=np.exp(y_log_lengthscales),
                y_sigma_n_init=float(np.exp(y_log_sigma_n)), x_lambdas_init=np.exp(x_log_lambdas),
                x_lengthscales_init=np.exp(x_log_lengthscales), x_sigma_n_init=float(np.exp(x_log_sigma_n)),
                x_lin_coeff_init=np.exp(x_log_lin_coeff), sigma_n_num_X=sigma_n_num_X,
                sigma_n_num_Y=sigma_n_num_Y, device=device)
        # keep the exact log parameters (exp/log round trips can move an ulp)
        m._set_param("y_log_lengthscales", np.asarray(y_log_lengthscales, dtype=np.float64))
        m._set_param("y_log_lambdas", np.asarray(y_log_lambdas, dtype=np.float64))
        m._set_param("y_log_sigma_n", np.float64(y_log_sigma_n))
        m._set_param("x_log_lengthscales", np.asarray(x_log_lengthscales, dtype=np.float64))
        m._set_param("x_log_lambdas", np.asarray(x_log_lambdas, dtype=np.float64))
        m._set_param("x_log_sigma_n", np.float64(x_log_sigma_n))
        m._set_param("x_log_lin_coeff", np.asarray(x_log_lin_coeff, dtype=np.float64))
        for c, seqs in enumerate(Y_sequences):
            for y in seqs:
                m.add_data(np.asarray(y), c)
        m.set_latents(X)
        return m
