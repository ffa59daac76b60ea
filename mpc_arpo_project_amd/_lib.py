"""ctypes binding of libmpcqp.so (the C ABI declared in include/mpcqp.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc --offload-arch=gfx950).  There is
no fallback: if the shared object is missing, or no GPU is visible when a device call is made, the
calls raise `MPCQPError`.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPCQP_LIBRARY selects another build of the same ABI (diagnostic builds in tools/), honoured only
# together with MPCQP_DIAGNOSTICS=1 like every other MPCQP_* override (csrc/symbolic.hpp diag_env);
# there is no fallback to anything else
_DIAG = os.environ.get("MPCQP_DIAGNOSTICS") == "1"
if os.environ.get("MPCQP_LIBRARY") and not _DIAG:
    # an A/B script that forgot the second variable would otherwise measure the product library
    raise RuntimeError("MPCQP_LIBRARY is set without MPCQP_DIAGNOSTICS=1: diagnostic libraries "
                       "load only under MPCQP_DIAGNOSTICS=1")
LIB_PATH = (_DIAG and os.environ.get("MPCQP_LIBRARY")) or os.path.join(_HERE, "libmpcqp.so")



def source_digest():
    """First 12 hex digits of a sha256 over the sources libmpcqp.so is built from (csrc/ and
    include/, sorted by name).  tools/profile_post.py stamps it into the committed profiles and
    bench.py compares it with the tree it runs from, so a profile is matched to the benched build
    by content, not only by the commit it was measured at."""
    import hashlib

    h = hashlib.sha256()
    repo = os.path.dirname(_HERE)
    for d in (os.path.join(_HERE, "csrc"), os.path.join(repo, "include")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".cpp", ".hpp", ".inc", ".h")):
                h.update(f.encode())
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:12]


# every symbol include/mpcqp.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "mpcqp_default_settings", "mpcqp_create", "mpcqp_destroy", "mpcqp_set_data",
    "mpcqp_update_bounds", "mpcqp_update_A", "mpcqp_update_lin_cost", "mpcqp_warm_start",
    "mpcqp_solve", "mpcqp_data_buffers", "mpcqp_copy_data", "mpcqp_set_skip", "mpcqp_set_order", "mpcqp_get_state", "mpcqp_set_state", "mpcqp_get_scaling", "mpcqp_dims", "mpcqp_schedule_info", "mpcqp_analyze", "mpcqp_export_symbolic",
    "mpcqp_schedule_check", "mpcqp_emu_create", "mpcqp_emu_clone", "mpcqp_emu_destroy", "mpcqp_emu_factor",
    "mpcqp_emu_solve",
    "mpcqp_status_string", "mpcqp_last_error", "mpcqp_version", "mpcqp_engine_kind", "mpcqp_schedule_kind",
    "mpcqp_kernel_info",
    "mpcqp_cl_create", "mpcqp_cl_destroy", "mpcqp_cl_configure", "mpcqp_cl_step",
    "mpcqp_cl_set_ids", "mpcqp_cl_set_tracking", "mpcqp_cl_noise", "mpcqp_cl_set_plant", "mpcqp_clc_period",
    "mpcqp_ukf_create", "mpcqp_ukf_destroy", "mpcqp_ukf_step", "mpcqp_plant_rk45",
)

STATUS = {
    1: "solved", 2: "solved inaccurate", 3: "primal infeasible inaccurate",
    4: "dual infeasible inaccurate", -2: "maximum iterations reached", -3: "primal infeasible",
    -4: "dual infeasible", -5: "interrupted", -6: "run time limit reached",
    -7: "problem non convex", -10: "unsolved",
}


class MPCQPError(RuntimeError):
    pass


class Structure(C.Structure):
    _fields_ = [("n", C.c_int32), ("m", C.c_int32),
                ("Pp", C.POINTER(C.c_int32)), ("Pi", C.POINTER(C.c_int32)),
                ("Ap", C.POINTER(C.c_int32)), ("Ai", C.POINTER(C.c_int32))]


class Settings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double),
        ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("delta", C.c_double), ("adaptive_rho_tolerance", C.c_double),
        ("max_iter", C.c_int32), ("scaling", C.c_int32), ("adaptive_rho", C.c_int32),
        ("adaptive_rho_interval", C.c_int32), ("polish", C.c_int32),
        ("polish_refine_iter", C.c_int32), ("check_termination", C.c_int32),
        ("warm_start", C.c_int32), ("scaled_termination", C.c_int32),
    ]


class Info(C.Structure):
    _fields_ = [("status", C.c_void_p), ("iter", C.c_void_p), ("rho_updates", C.c_void_p),
                ("obj_val", C.c_void_p), ("pri_res", C.c_void_p), ("dua_res", C.c_void_p),
                ("rho", C.c_void_p)]


class ClScenario(C.Structure):
    _fields_ = [
        ("Nx", C.c_int32), ("Nc", C.c_int32), ("Nb", C.c_int32), ("m", C.c_int32),
        ("nnzA", C.c_int32),
        ("Ad", C.c_double * 16), ("Bd", C.c_double * 8),
        ("rp", C.c_double), ("rtol", C.c_double), ("xr", C.c_double * 4),
        ("inTrack", C.c_int32), ("isReject", C.c_int32), ("has_debris", C.c_int32),
        ("center", C.c_double * 2), ("side", C.c_double), ("detect", C.c_double),
        ("verts", C.c_double * 8), ("umin", C.c_double * 7), ("umax", C.c_double * 7),
        ("Kpf", C.c_double * 8), ("Kif", C.c_double * 2), ("Ktot", C.c_double * 8),
        ("Ki", C.c_double * 2), ("Crefx", C.c_double * 4), ("Crefy", C.c_double * 4),
        ("pos_c1", C.POINTER(C.c_int32)), ("pos_c2", C.POINTER(C.c_int32)),
        ("pos_slope", C.POINTER(C.c_int32)),
    ]


class UkfModel(C.Structure):
    _fields_ = [("Ao", C.c_double * 36), ("Bou", C.c_double * 12), ("Q", C.c_double * 36),
                ("R", C.c_double * 4), ("alpha", C.c_double), ("beta", C.c_double),
                ("kappa", C.c_double)]


class PlantModel(C.Structure):
    _fields_ = [("two_n", C.c_double), ("m_two_n", C.c_double), ("n2", C.c_double),
                ("R_T", C.c_double), ("mu", C.c_double), ("g0", C.c_double),
                ("rtol", C.c_double), ("atol", C.c_double)]


_lib = None


def lib():
    """Load libmpcqp.so (raises MPCQPError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MPCQPError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    # a host-only build (no HIP: the planner, the schedule interpreter and the settings/status entry
    # points, for the sanitizer check of the host code, tests/test_sanitize.py) exports the marker
    # mpcqp_host_only_build and nothing that touches a GPU; the product library must export all
    host_only = hasattr(L, "mpcqp_host_only_build")
    # a diagnostic library of an earlier revision (MPCQP_LIBRARY, A/B runs) may predate a
    # white-box entry point; the product library must export every symbol
    diag_lib = LIB_PATH != os.path.join(_HERE, "libmpcqp.so")

    def _sig(L, name, what, value):
        fn = getattr(L, name, None)
        if fn is None:
            if host_only or (diag_lib and name in ("mpcqp_get_scaling",)):
                return
            raise MPCQPError(f"{LIB_PATH} does not export {name}")
        setattr(fn, what, value)

    vp, i32, i32p, dp = C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.c_void_p
    _sig(L, "mpcqp_default_settings", "argtypes", [C.POINTER(Settings)])
    _sig(L, "mpcqp_create", "argtypes", [C.POINTER(Structure), C.POINTER(Settings), i32, vp,
                               C.POINTER(vp)])
    _sig(L, "mpcqp_destroy", "argtypes", [vp])
    _sig(L, "mpcqp_set_data", "argtypes", [vp, dp, dp, dp, dp, dp])
    _sig(L, "mpcqp_update_bounds", "argtypes", [vp, dp, dp])
    _sig(L, "mpcqp_update_A", "argtypes", [vp, dp])
    _sig(L, "mpcqp_update_lin_cost", "argtypes", [vp, dp])
    _sig(L, "mpcqp_warm_start", "argtypes", [vp, dp, dp])
    _sig(L, "mpcqp_solve", "argtypes", [vp, dp, dp, C.POINTER(Info)])
    _sig(L, "mpcqp_dims", "argtypes", [vp, i32p, i32p, i32p, i32p, i32p])
    _sig(L, "mpcqp_engine_kind", "argtypes", [vp, i32p])
    _sig(L, "mpcqp_schedule_kind", "argtypes", [vp, i32p])
    _sig(L, "mpcqp_kernel_info", "argtypes", [vp, i32p, i32p, i32p, i32p])
    _sig(L, "mpcqp_copy_data", "argtypes", [vp, dp, dp, dp])
    _sig(L, "mpcqp_get_state", "argtypes", [vp, dp, dp, dp, dp, dp])
    _sig(L, "mpcqp_set_state", "argtypes", [vp, dp, dp, dp, dp, dp])
    _sig(L, "mpcqp_get_scaling", "argtypes", [vp, dp, dp, dp])
    _sig(L, "mpcqp_set_skip", "argtypes", [vp, dp])
    _sig(L, "mpcqp_set_order", "argtypes", [vp, dp])
    _sig(L, "mpcqp_data_buffers", "argtypes", [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)])
    _sig(L, "mpcqp_schedule_info", "argtypes", [vp, i32p, i32p, i32p, i32p, i32p])
    _sig(L, "mpcqp_export_symbolic", "argtypes", [vp, i32p, i32p, i32p])
    _sig(L, "mpcqp_analyze", "argtypes", [C.POINTER(Structure), i32p, i32p, i32p, i32p, i32p])
    _sig(L, "mpcqp_schedule_check", "argtypes", [C.POINTER(Structure), dp, dp, C.c_double, dp, dp, dp,
                                       C.POINTER(C.c_int64)])
    _sig(L, "mpcqp_emu_create", "argtypes", [C.POINTER(Structure), C.POINTER(vp)])
    _sig(L, "mpcqp_emu_clone", "argtypes", [vp, C.POINTER(vp)])
    _sig(L, "mpcqp_emu_destroy", "argtypes", [vp])
    _sig(L, "mpcqp_emu_factor", "argtypes", [vp, dp, dp, C.c_double, dp])
    _sig(L, "mpcqp_emu_solve", "argtypes", [vp, dp, dp])
    _sig(L, "mpcqp_cl_create", "argtypes", [C.POINTER(ClScenario), i32, vp, C.POINTER(vp)])
    _sig(L, "mpcqp_cl_destroy", "argtypes", [vp])
    _sig(L, "mpcqp_cl_configure", "argtypes", [vp, dp, dp, dp, dp])
    _sig(L, "mpcqp_cl_step", "argtypes", [vp, dp, dp, i32, i32, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp])
    _sig(L, "mpcqp_cl_set_ids", "argtypes", [vp, C.c_int64])
    _sig(L, "mpcqp_cl_set_tracking", "argtypes", [vp, dp, dp, dp, dp, C.c_double, C.c_double])
    _sig(L, "mpcqp_cl_noise", "argtypes", [vp, C.c_uint64, C.c_uint64, C.c_double, C.c_double, dp])
    _sig(L, "mpcqp_cl_set_plant", "argtypes", [vp, C.POINTER(PlantModel), i32])
    _sig(L, "mpcqp_clc_period", "argtypes", [vp, dp, dp, i32, i32, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp,
                                   dp, C.c_double, C.c_double, i32, i32, dp])
    _sig(L, "mpcqp_ukf_create", "argtypes", [C.POINTER(UkfModel), i32, vp, C.POINTER(vp)])
    _sig(L, "mpcqp_ukf_destroy", "argtypes", [vp])
    _sig(L, "mpcqp_ukf_step", "argtypes", [vp, dp, dp, dp, dp, dp, dp])
    _sig(L, "mpcqp_plant_rk45", "argtypes", [C.POINTER(PlantModel), i32, vp, dp, dp, dp, C.c_double,
                                   C.c_double, i32, dp, dp])
    _sig(L, "mpcqp_status_string", "argtypes", [i32])
    _sig(L, "mpcqp_status_string", "restype", C.c_char_p)
    _sig(L, "mpcqp_last_error", "restype", C.c_char_p)
    for name in EXPORTED:
        fn = getattr(L, name, None)
        if fn is None:
            continue  # host-only diagnostics build (checked by _sig)
        if name not in ("mpcqp_status_string", "mpcqp_last_error"):
            fn.restype = C.c_int
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().mpcqp_last_error().decode(errors="replace")
        raise MPCQPError(f"{what} failed ({rc}): {msg}")


def default_settings(**overrides) -> Settings:
    s = Settings()
    lib().mpcqp_default_settings(C.byref(s))
    for k, v in overrides.items():
        if k == "verbose":
            continue
        if k == "warm_starting":  # OSQP 1.x spelling
            k = "warm_start"
        if not any(k == f[0] for f in Settings._fields_):
            raise ValueError(f"unknown setting '{k}'")
        setattr(s, k, type(getattr(s, k))(v))
    return s


def analyze(P_triu_csc, A_csc):
    """Host-only symbolic analysis (no GPU): perm, Lp, Li and schedule statistics."""
    import numpy as np

    n, m = P_triu_csc.shape[0], A_csc.shape[0]
    Pp = np.ascontiguousarray(P_triu_csc.indptr, dtype=np.int32)
    Pi = np.ascontiguousarray(P_triu_csc.indices, dtype=np.int32)
    Ap = np.ascontiguousarray(A_csc.indptr, dtype=np.int32)
    Ai = np.ascontiguousarray(A_csc.indices, dtype=np.int32)
    i32 = C.POINTER(C.c_int32)
    st = Structure(n, m, Pp.ctypes.data_as(i32), Pi.ctypes.data_as(i32), Ap.ctypes.data_as(i32),
                   Ai.ctypes.data_as(i32))
    perm = np.empty(n + m, dtype=np.int32)
    Lp = np.empty(n + m + 1, dtype=np.int32)
    nnz = C.c_int32(0)
    stats = np.empty(6, dtype=np.int32)
    check(lib().mpcqp_analyze(C.byref(st), perm.ctypes.data_as(i32), Lp.ctypes.data_as(i32), None,
                              C.byref(nnz), stats.ctypes.data_as(i32)), "mpcqp_analyze")
    Li = np.empty(max(nnz.value, 1), dtype=np.int32)
    check(lib().mpcqp_analyze(C.byref(st), None, None, Li.ctypes.data_as(i32), C.byref(nnz), None),
          "mpcqp_analyze")
    keys = ("fac_steps", "fwd_steps", "bwd_steps", "fwd_levels", "bwd_levels", "lds_image_bytes")
    return perm, Lp, Li[:nnz.value], dict(zip(keys, stats.tolist()))


def schedule_check(P_triu_csc, A_csc, sigma, rho_vec, rhs):
    """Host-only (no GPU): the compiled device program interpreted on the CPU for one instance
    (assembly, factorization, one KKT solve).  Returns (solution of the KKT system for rhs,
    modelled LDS cycles dict).  Test / diagnostic use."""
    import numpy as np

    n, m = P_triu_csc.shape[0], A_csc.shape[0]
    Pp = np.ascontiguousarray(P_triu_csc.indptr, dtype=np.int32)
    Pi = np.ascontiguousarray(P_triu_csc.indices, dtype=np.int32)
    Ap = np.ascontiguousarray(A_csc.indptr, dtype=np.int32)
    Ai = np.ascontiguousarray(A_csc.indices, dtype=np.int32)
    i32 = C.POINTER(C.c_int32)
    d = C.POINTER(C.c_double)
    st = Structure(n, m, Pp.ctypes.data_as(i32), Pi.ctypes.data_as(i32), Ap.ctypes.data_as(i32),
                   Ai.ctypes.data_as(i32))
    Px = np.ascontiguousarray(P_triu_csc.data, dtype=np.float64)
    Ax = np.ascontiguousarray(A_csc.data, dtype=np.float64)
    rho = np.ascontiguousarray(rho_vec, dtype=np.float64)
    b = np.ascontiguousarray(rhs, dtype=np.float64)
    sol = np.empty(n + m, dtype=np.float64)
    model = np.zeros(4, dtype=np.int64)
    check(lib().mpcqp_schedule_check(C.byref(st), Px.ctypes.data_as(d), Ax.ctypes.data_as(d),
                                     float(sigma), rho.ctypes.data_as(d), b.ctypes.data_as(d),
                                     sol.ctypes.data_as(d), model.ctypes.data_as(C.POINTER(C.c_int64))),
          "mpcqp_schedule_check")
    return sol, dict(zip(("read", "atomic", "vec", "floor"), model.tolist()))
