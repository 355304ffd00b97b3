"""ctypes binding of libsnakehip.so (the C ABI in include/snakehip.h).

The shared library is the product: every computation of this package runs in
it on the GPU. There is no CPU fallback; if the library is missing or no HIP
device is visible, calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SNK_LIB: an alternative build of the same library (tools/ profiling variants)
LIB_PATH = os.environ.get("SNK_LIB") or os.path.join(_HERE, "libsnakehip.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "snakehip.h")

SNK_OK = 0
SNK_ERR_INVALID = 1
SNK_ERR_FOOD_EXHAUSTED = 2
SNK_ERR_HIP = 3
SNK_ERR_NOMEM = 4
SNK_ERR_STATE = 5
SNK_ERR_INTERNAL = 6
SNK_ACT_INDEX = 0
SNK_ACT_DIRECTION = 1


class SnakeHipError(RuntimeError):
    """A non-zero status from libsnakehip."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[snk status {code}] {msg}")
        self.code = code


class FoodListExhausted(SnakeHipError):
    """The reference throws BoundsError here (utils.jl:37 `board[0] = 2`)."""


class BufferSizeError(SnakeHipError):
    """structs.jl:113 `batch_size cannot be greater than the capacity of the buffer.`"""


_lib = None

vp = C.c_void_p
i32, i64, u32, u64, f32, f64 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_float, C.c_double
P = C.POINTER

# name -> argtypes (restype is int status unless listed in _RESTYPE)
_PROTOS = {
    "snk_last_error": [],
    "snk_version": [P(i32)],
    "snk_build_source_sha256": [],
    "snk_device_count": [P(i32)],
    "snk_set_device": [i32],
    "snk_set_stream": [vp],
    "snk_synchronize": [],
    "snk_set_arith": [i32, i32],
    "snk_get_arith": [i32, P(i32)],
    "snk_malloc": [P(vp), i64],
    "snk_free": [vp],
    "snk_memcpy_h2d": [vp, vp, i64],
    "snk_memcpy_d2h": [vp, vp, i64],
    "snk_memset": [vp, i32, i64],
    "snk_food_list": [i32, u32, i32, vp],
    "snk_env_create": [P(vp), i64, i32, i32, u32, i32, i32],
    "snk_env_destroy": [vp],
    "snk_env_reset": [vp, vp],
    "snk_env_step": [vp, vp, i32],
    "snk_env_outputs": [vp, P(vp), P(vp), P(vp), P(vp), P(vp), P(vp)],
    "snk_env_get_boards": [vp, vp],
    "snk_env_get_states": [vp, vp],
    "snk_env_get_scalars": [vp, vp, vp, vp, vp, vp, vp],
    "snk_env_get_snake": [vp, i64, vp, P(i32)],
    "snk_env_check_faults": [vp, P(i64)],
    "snk_env_synth_actions": [vp, u64, vp],
    "snk_env_info": [vp, P(i64), P(i32), P(i32), P(i64)],
    "snk_replay_create": [P(vp), i64, i32, i32, i32],
    "snk_replay_destroy": [vp],
    "snk_env_step_store": [vp, vp, i32, vp],
    "snk_replay_store": [vp, i64, vp, vp, vp, vp, vp, vp],
    "snk_replay_length": [vp, P(i64)],
    "snk_replay_position": [vp, P(i64)],
    "snk_replay_empty": [vp],
    "snk_replay_sample": [vp, u64, u64, vp, P(i32)],
    "snk_replay_gather": [vp, vp, i64, vp, vp, vp, vp, vp, vp, vp],
    "snk_dqn_create": [P(vp), i32, i32, f32, f32, f32, u64],
    "snk_dqn_destroy": [vp],
    "snk_dqn_create_deep": [P(vp), i32, i32, f32, f32, f32, u64],
    "snk_dqn_time_deep_layers": [vp, vp, i32, vp],
    "snk_dqn_nparams": [vp, P(i64)],
    "snk_dqn_set_params": [vp, i32, vp],
    "snk_dqn_get_params": [vp, i32, vp],
    "snk_dqn_buffer_ptr": [vp, i32, P(vp)],
    "snk_dqn_sync_target": [vp],
    "snk_dqn_forward": [vp, i32, vp, i64, vp],
    "snk_dqn_forward_env": [vp, i32, vp, vp],
    "snk_dqn_act": [vp, vp, f32, u64, vp],
    "snk_dqn_last_q": [vp, vp, i64],
    "snk_dqn_time_act_layers": [vp, vp, i32, vp],
    "snk_env_time_step": [vp, vp, vp, i32, P(f64)],
    "snk_dqn_train_activations": [vp, i32, vp, i64],
    "snk_dqn_loss_grad": [vp, vp, vp, i64, f64, P(f64)],
    "snk_dqn_loss_grad_batch": [vp, vp, vp, vp, vp, vp, vp, i64, f64, P(f64)],
    "snk_dqn_apply_grad": [vp],
    "snk_dqn_update": [vp, vp, vp, i64, f64, P(f64)],
    "snk_abi_sizes": [P(i64), P(i64)],
    "snk_trainer_create": [P(vp), vp, vp, vp, vp],
    "snk_trainer_destroy": [vp],
    "snk_trainer_run": [vp, i64, i32, i32],
    "snk_trainer_run_partial": [vp, i32],
    "snk_trainer_set_nb": [vp, i64],
    "snk_trainer_set_trace": [vp, vp, i64],
    "snk_trainer_set_act_trace": [vp, vp, vp, i64],
    "snk_trainer_stats": [vp, vp],
    "snk_trainer_time_act_kernel": [vp, i32, vp],
    "snk_trainer_losses": [vp, vp, i64],
    "snk_trainer_act_ptr": [vp, P(vp)],
    "snk_trainer_set_comm": [vp, vp],
    "snk_comm_unique_id": [vp],
    "snk_comm_create": [P(vp), i32, i32, vp],
    "snk_comm_destroy": [vp],
    "snk_comm_allreduce_mean": [vp, vp, i64],
    "snk_comm_broadcast": [vp, vp, i64, i32],
    "snk_comm_info": [vp, P(i32), P(i32)],
    "snk_laplace_create": [P(vp), i64, i32],
    "snk_laplace_destroy": [vp],
    "snk_laplace_snapshot": [vp, vp, i32],
    "snk_laplace_set_column": [vp, i32, vp],
    "snk_laplace_get": [vp, i32, vp, i64],
    "snk_laplace_buffer_ptr": [vp, i32, P(vp), P(i64)],
    "snk_laplace_fit_center": [vp],
    "snk_laplace_gram": [vp, P(f32)],
    "snk_jacobian": [vp, vp, vp, i64, vp],
    "snk_jacobian_gram": [vp, vp, i64, vp, P(f32)],
    "snk_jacobian_gram_shard": [vp, vp, i64, i32, i32, vp, P(f32)],
    "snk_gram_tiles": [i64, i32, i32, vp, P(i64)],
    "snk_jacobian_gram_gather": [vp, i64, vp, i32],
    "snk_laplace_normals": [u64, i64, i32, i64, i64, vp],
    "snk_laplace_sample_params": [vp, vp, u64, i64, vp],
    "snk_laplace_sampling": [vp, vp, vp, i64, u64, i64, P(f32), P(i64), vp, vp],
}

SNK_NET_Q = 0
SNK_NET_TARGET = 1
SNK_NET_OPT_STATE = 2
SNK_NET_GRAD = 3
SNK_LAP_D = 0
SNK_LAP_MEAN = 1
SNK_LAP_VAR = 2
SNK_LAP_GRAM = 3
SNK_LAP_D32 = 4


class TrainerCfg(C.Structure):
    """snk_trainer_cfg_t (struct_size set by the constructor: the library's ABI guard)"""
    _fields_ = [("struct_size", i32), ("epsilon", f32), ("epsilon_end", f32), ("decay", f32), ("updates_per_iter", i32),
                ("target_update_rate", i64), ("gamma", f64), ("seed", u64), ("loss_log_capacity", i64),
                ("graph_unroll", i32)]

    def __init__(self, *args, **kw):
        super().__init__(C.sizeof(self), *args, **kw)


class TrainerStats(C.Structure):
    """snk_trainer_stats_t (struct_size set by the constructor: the library's ABI guard)"""
    _fields_ = [("struct_size", i32), ("episodes", i64), ("score_sum", i64), ("updates", i64), ("nb", i64), ("env_steps", i64),
                ("reward_sum", f64), ("last_loss", f64), ("reward_max", f32), ("score_max", i32),
                ("epsilon", f32)]

    def __init__(self, *args, **kw):
        super().__init__(C.sizeof(self), *args, **kw)


_RESTYPE = {"snk_last_error": C.c_char_p, "snk_build_source_sha256": C.c_char_p}


def header_symbols() -> list[str]:
    """Every function the C header declares (used by the ABI test)."""
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(snk_[a-z0-9_]+)\s*\(", txt)))


def load():
    """Load libsnakehip.so. torch is imported first when present so that the
    process holds ONE HIP runtime (torch ships its own libamdhip64)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional plumbing
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIB_PATH)
    for name, args in _PROTOS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, C.c_int)
    _lib = lib
    return lib


def source_sha256(csrc: str | None = None) -> str:
    """The build-provenance hash of a source tree, as csrc/Makefile computes it
    (`sha256sum $(sort *.hip *.hpp ../../include/snakehip.h Makefile) | sha256sum`)."""
    import glob
    import hashlib
    csrc = csrc or os.path.join(_HERE, "csrc")
    names = [os.path.basename(f) for f in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))]
    names += ["../../include/snakehip.h", "Makefile"]
    lines = ""
    for n in sorted(names):
        with open(os.path.join(csrc, n), "rb") as f:
            lines += f"{hashlib.sha256(f.read()).hexdigest()}  {n}\n"
    return hashlib.sha256(lines.encode()).hexdigest()


def build_provenance() -> dict:
    """Which sources the loaded library was linked from, against the tree beside it."""
    lib_h = load().snk_build_source_sha256().decode()
    tree_h = source_sha256()
    return {"lib": os.path.basename(LIB_PATH), "lib_source_sha256": lib_h, "tree_source_sha256": tree_h,
            "lib_matches_tree": lib_h == tree_h}


def check(status: int):
    if status == SNK_OK:
        return
    msg = load().snk_last_error().decode(errors="replace")
    if status == SNK_ERR_FOOD_EXHAUSTED:
        raise FoodListExhausted(status, msg)
    if status == SNK_ERR_STATE and "capacity" in msg:
        raise BufferSizeError(status, msg)
    raise SnakeHipError(status, msg)


def call(name: str, *args):
    check(getattr(load(), name)(*args))


def ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "host arrays must be C-contiguous"
    return a.ctypes.data_as(vp)


def header_arith() -> dict[str, int]:
    """snk_set_arith knobs as the header defines them: SNK_ARITH_<NAME> -> name.lower()."""
    with open(HEADER) as f:
        txt = f.read()
    return {m.group(1).lower(): int(m.group(2))
            for m in re.finditer(r"#define\s+SNK_ARITH_(\w+)\s+(\d+)", txt) if m.group(1) != "COUNT"}


# snk_set_arith knobs (include/snakehip.h SNK_ARITH_*): name -> knob
ARITH = header_arith()


def set_arith(name: str, value: bool) -> bool:
    """Select a GEMM arithmetic path process-wide (SNK_ARITH_*); returns the previous
    value. Production defaults: x6s, h3s, dh3, h3c2, upd_head, env_head, split_chain, syrk_ksplit on;
    conv_fp32, syrk_h3_32 off."""
    old = get_arith(name)
    call("snk_set_arith", ARITH[name], int(bool(value)))
    return old


def get_arith(name: str) -> bool:
    v = i32(0)
    call("snk_get_arith", ARITH[name], C.byref(v))
    return bool(v.value)


class arith:
    """Context manager: `with arith(dh3=False): ...` runs the block on the
    comparison path and restores the previous selection."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.old = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.old[k] = set_arith(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_arith(k, v)
        return False


def device_count() -> int:
    n = i32(0)
    try:
        call("snk_device_count", C.byref(n))
    except SnakeHipError:
        return 0
    return n.value


class DeviceArray:
    """A device allocation owned by the library allocator (snk_malloc)."""

    def __init__(self, shape, dtype):
        self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = vp()
        call("snk_malloc", C.byref(p), max(self.nbytes, 1))
        self.ptr = p

    @classmethod
    def from_host(cls, a: np.ndarray):
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        d.upload(a)
        return d

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a, self.dtype)
        assert a.nbytes == self.nbytes, (a.nbytes, self.nbytes)
        call("snk_memcpy_h2d", self.ptr, ptr(a), self.nbytes)

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        call("snk_memcpy_d2h", ptr(out), self.ptr, self.nbytes)
        return out

    def zero(self):
        call("snk_memset", self.ptr, 0, self.nbytes)

    def __del__(self):
        if getattr(self, "ptr", None) and self.ptr.value and _lib is not None:
            _lib.snk_free(self.ptr)
            self.ptr = None


def view_numpy(dev_ptr: int, shape, dtype) -> np.ndarray:
    """Copy `shape` elements at a raw device pointer to a new host array."""
    out = np.empty(shape, dtype)
    call("snk_memcpy_d2h", ptr(out), vp(dev_ptr), out.nbytes)
    return out
