"""ctypes binding of the go2pi C ABI (include/go2pi.h) -> `Engine`.

The shared library is built in-tree (go2_onnx_controller_amd/lib/libgo2pi.so,
see __graft_entry__.build()). There is deliberately NO CPU fallback: if the
library or a HIP device is missing, construction raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
LIB_PATH = os.environ.get("GO2PI_LIB") or os.path.join(LIB_DIR, "libgo2pi.so")  # override: diagnostics only
ACTOR_LIB_PATH = os.path.join(LIB_DIR, "libonnx_actor.so")

# every symbol include/go2pi.h declares (tests check the .so exports them all)
EXPORTS = [
    "go2pi_default_opts", "go2pi_create", "go2pi_create_from_memory", "go2pi_destroy", "go2pi_num_io",
    "go2pi_io_name", "go2pi_io_shape", "go2pi_io_dims", "go2pi_run", "go2pi_run_device",
    "go2pi_run_sequence_device", "go2pi_reset_hidden", "go2pi_get_hidden", "go2pi_set_hidden",
    "go2pi_hidden_dim", "go2pi_sync", "go2pi_get_cost", "go2pi_batched_kernel", "go2pi_inspect_model",
    "go2pi_diag_stamps", "go2pi_resident_kernel", "go2pi_resident_launches",
    "go2pi_last_error", "go2pi_version", "go2pi_ctl_default_params", "go2pi_ctl_set_params",
    "go2pi_ctl_history", "go2pi_controller_step", "go2pi_controller_step_device",
]

# controller tick row layouts (include/go2pi.h GO2PI_CTL_*)
CTL_STATE_DIM = 36
CTL_JOY_DIM = 5
CTL_DOF = 12

GO2PI_OK = 0
ERRORS = {-1: "GO2PI_E_INVALID", -2: "GO2PI_E_MODEL", -3: "GO2PI_E_DEVICE", -4: "GO2PI_E_CAPACITY"}


class Go2piError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Opts(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("max_batch", ctypes.c_int64),
        ("use_graph", ctypes.c_int32),
        ("log_level", ctypes.c_int32),
        ("waves", ctypes.c_int32),
        ("small_batch", ctypes.c_int32),
        ("obs_mean", ctypes.c_void_p),
        ("obs_std", ctypes.c_void_p),
        ("obs_clip", ctypes.c_float),
        ("action_tanh", ctypes.c_int32),
        ("action_clip", ctypes.c_float),
        ("action_scale", ctypes.c_float),
        ("resident_ms", ctypes.c_int32),
    ]


class Cost(ctypes.Structure):
    _fields_ = [
        ("flops_per_row", ctypes.c_double),
        ("weight_bytes", ctypes.c_double),
        ("io_bytes_per_row", ctypes.c_double),
        ("n_layers", ctypes.c_int32),
        ("has_gru", ctypes.c_int32),
    ]


class CtlParams(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_int32),
        ("kp", ctypes.c_float),
        ("kd", ctypes.c_float),
        ("kp_stop", ctypes.c_float),
        ("action_limit", ctypes.c_float),
        ("contact_threshold", ctypes.c_float),
        ("gravity_w", ctypes.c_float * 3),
        ("action_scale", ctypes.c_double),
        ("q0", ctypes.c_double * 12),
    ]


_lib = None


def lib():
    """Load libgo2pi.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        # Share ONE HIP runtime with PyTorch: torch bundles its own libamdhip64.so
        # (same SONAME). Loading torch first makes our NEEDED libamdhip64.so.7 bind to
        # it, so torch streams / device pointers are valid handles for go2pi.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        sig = {
            "go2pi_default_opts": (None, [P]),
            "go2pi_create": (ctypes.c_int, [ctypes.c_char_p, P, P]),
            "go2pi_create_from_memory": (ctypes.c_int, [P, ctypes.c_size_t, P, P]),
            "go2pi_destroy": (None, [P]),
            "go2pi_num_io": (ctypes.c_int, [P, P, P]),
            "go2pi_io_name": (ctypes.c_int, [P, I32, I32, ctypes.c_char_p, ctypes.c_size_t]),
            "go2pi_io_shape": (ctypes.c_int, [P, I32, I32, P, I32, P]),
            "go2pi_io_dims": (ctypes.c_int, [P, P, P]),
            "go2pi_run": (ctypes.c_int, [P, P, P, I64]),
            "go2pi_run_device": (ctypes.c_int, [P, P, P, I64, P]),
            "go2pi_run_sequence_device": (ctypes.c_int, [P, P, P, I64, I64, P]),
            "go2pi_reset_hidden": (ctypes.c_int, [P, P, I64]),
            "go2pi_get_hidden": (ctypes.c_int, [P, P, I64]),
            "go2pi_set_hidden": (ctypes.c_int, [P, P, I64]),
            "go2pi_hidden_dim": (ctypes.c_int, [P, P]),
            "go2pi_sync": (ctypes.c_int, [P]),
            "go2pi_get_cost": (ctypes.c_int, [P, P]),
            "go2pi_batched_kernel": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.c_size_t]),
            "go2pi_resident_kernel": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.c_size_t]),
            "go2pi_resident_launches": (ctypes.c_int, [P, P]),
            "go2pi_diag_stamps": (ctypes.c_int, [P, P, I64]),
            "go2pi_inspect_model": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
            "go2pi_last_error": (ctypes.c_char_p, []),
            "go2pi_version": (ctypes.c_char_p, []),
            "go2pi_ctl_default_params": (None, [P]),
            "go2pi_ctl_set_params": (ctypes.c_int, [P, P]),
            "go2pi_ctl_history": (ctypes.c_int, [P, P]),
            "go2pi_controller_step": (ctypes.c_int, [P, P, P, P, P, P, P, P, P, I64]),
            "go2pi_controller_step_device": (ctypes.c_int, [P, P, P, P, P, P, P, P, P, I64, P]),
        }
        for name, (res, args) in sig.items():
            if name in ("go2pi_batched_kernel", "go2pi_resident_kernel", "go2pi_resident_launches") and not hasattr(L, name) and \
                    os.environ.get("GO2PI_LIB"):
                continue  # an older diagnostics build (A/B tooling): the name query is optional there
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != GO2PI_OK:
        raise Go2piError(rc, lib().go2pi_last_error().decode(errors="replace"))


def _f32(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} floats, got {a.size}")
    return a


class Engine:
    """One loaded policy on one GPU. Not thread-safe per instance (like ONNXActor)."""

    def __init__(self, model, device=0, max_batch=4096, use_graph=True, waves=0, small_batch=0,
                 obs_mean=None, obs_std=None, obs_clip=0.0, action_tanh=False, action_clip=0.0,
                 action_scale=0.0, log_level=2, resident_ms=0):
        L = lib()
        o = Opts()
        L.go2pi_default_opts(ctypes.byref(o))
        o.device, o.max_batch, o.use_graph = int(device), int(max_batch), int(bool(use_graph))
        o.waves, o.small_batch, o.log_level = int(waves), int(small_batch), int(log_level)
        self._keep = []
        if obs_mean is not None:
            m = _f32(obs_mean)
            self._keep.append(m)
            o.obs_mean = m.ctypes.data
        if obs_std is not None:
            s = _f32(obs_std)
            self._keep.append(s)
            o.obs_std = s.ctypes.data
        o.obs_clip, o.action_tanh = float(obs_clip), int(bool(action_tanh))
        o.action_clip, o.action_scale = float(action_clip), float(action_scale)
        o.resident_ms = int(resident_ms)  # > 0: batch <= 8 run() served by a resident kernel
        h = ctypes.c_void_p()
        if isinstance(model, (bytes, bytearray)):
            buf = bytes(model)
            _check(L.go2pi_create_from_memory(buf, len(buf), ctypes.byref(o), ctypes.byref(h)))
        else:
            _check(L.go2pi_create(os.fsencode(model), ctypes.byref(o), ctypes.byref(h)))
        self._h = h
        self.device = int(device)
        self.max_batch = int(max_batch)
        i, j = ctypes.c_int64(), ctypes.c_int64()
        _check(L.go2pi_io_dims(h, ctypes.byref(i), ctypes.byref(j)))
        self.in_dim, self.out_dim = i.value, j.value
        hd = ctypes.c_int64()
        _check(L.go2pi_hidden_dim(h, ctypes.byref(hd)))
        self.hidden_dim = hd.value
        ni, no = ctypes.c_int32(), ctypes.c_int32()
        _check(L.go2pi_num_io(h, ctypes.byref(ni), ctypes.byref(no)))
        self.inputs = [self._io(0, k) for k in range(ni.value)]
        self.outputs = [self._io(1, k) for k in range(no.value)]
        c = Cost()
        _check(L.go2pi_get_cost(h, ctypes.byref(c)))
        self.cost = {"flops_per_row": c.flops_per_row, "weight_bytes": c.weight_bytes,
                     "io_bytes_per_row": c.io_bytes_per_row, "n_layers": c.n_layers, "has_gru": bool(c.has_gru),
                     "cell": {0: None, 1: "GRU", 2: "LSTM"}.get(c.has_gru)}
        # recurrent state per robot: GRU h [H]; LSTM h [H] | c [H] (hidden_dim = their sum)
        self.batched_kernel = "unknown"
        if hasattr(L, "go2pi_batched_kernel") and L.go2pi_batched_kernel.argtypes:
            kb = ctypes.create_string_buffer(128)
            _check(L.go2pi_batched_kernel(h, kb, 128))
            self.batched_kernel = kb.value.decode()  # e.g. "policy_mlp_kernel<8, 1, 3, 1, 3, 4>" (rocprofv3 name)
        self.resident_kernel = "unknown"
        if hasattr(L, "go2pi_resident_kernel") and L.go2pi_resident_kernel.argtypes:
            kb = ctypes.create_string_buffer(128)
            _check(L.go2pi_resident_kernel(h, kb, 128))
            self.resident_kernel = kb.value.decode()  # e.g. "policy_wide_kernel<4, 8, 12, 0> ring=vram"

    @property
    def resident_launches(self):
        """Resident kernel launches so far (go2pi_resident_launches): one per idle-out,
        stop or abort; a kernel that gives up on every request shows as one per call."""
        n = ctypes.c_int64(0)
        _check(lib().go2pi_resident_launches(self._h, ctypes.byref(n)))
        return n.value

    def _io(self, is_out, k):
        L = lib()
        buf = ctypes.create_string_buffer(512)
        _check(L.go2pi_io_name(self._h, is_out, k, buf, 512))
        dims = (ctypes.c_int64 * 8)()
        rank = ctypes.c_int32()
        _check(L.go2pi_io_shape(self._h, is_out, k, dims, 8, ctypes.byref(rank)))
        return buf.value.decode(), [dims[d] for d in range(min(rank.value, 8))]

    # ----------------------------------------------------------- host path
    def run(self, obs, out=None):
        """obs [B, in_dim] (host) -> action [B, out_dim] float32 (host)."""
        x = _f32(obs)
        if x.ndim == 1:
            x = x.reshape(1, -1)
        if x.shape[-1] != self.in_dim:
            raise ValueError(f"observation feature dim {x.shape[-1]} != {self.in_dim}")
        B = x.shape[0]
        if out is None:
            out = np.empty((B, self.out_dim), np.float32)
        if not (out.flags.c_contiguous and out.dtype == np.float32 and out.size == B * self.out_dim):
            raise ValueError("out must be a C-contiguous float32 array of [B, out_dim]")
        _check(lib().go2pi_run(self._h, x.ctypes.data, out.ctypes.data, B))
        return out

    def run_ptr(self, obs_ptr, act_ptr, batch):
        """Host pointers, as ONNXActor::act() binds them (zero-copy aliasing)."""
        _check(lib().go2pi_run(self._h, obs_ptr, act_ptr, int(batch)))

    # --------------------------------------------------------- device path
    def run_device(self, obs_ptr, act_ptr, batch, stream=None):
        _check(lib().go2pi_run_device(self._h, obs_ptr, act_ptr, int(batch), stream))

    def device_launcher(self, obs_ptr, act_ptr, batch, stream=None):
        """Pre-bound zero-argument launcher for tight host loops: the ctypes
        arguments are converted once, so the per-call host cost is the C ABI's."""
        fn = lib().go2pi_run_device
        args = (self._h, ctypes.c_void_p(obs_ptr), ctypes.c_void_p(act_ptr), ctypes.c_int64(int(batch)),
                ctypes.c_void_p(stream))

        def launch():
            rc = fn(*args)
            if rc:
                _check(rc)
        return launch

    def run_sequence_device(self, obs_ptr, act_ptr, steps, batch, stream=None):
        _check(lib().go2pi_run_sequence_device(self._h, obs_ptr, act_ptr, int(steps), int(batch), stream))

    def run_torch(self, obs, out=None, stream=None):
        """torch device tensors (on this engine's GPU): obs [B, in] -> act [B, out].
        Enqueued on torch's current stream unless `stream` (a torch.cuda.Stream) is given."""
        import torch
        if obs.dtype != torch.float32 or not obs.is_contiguous() or obs.device.type != "cuda":
            raise ValueError("obs must be a contiguous float32 CUDA/HIP tensor")
        B = obs.shape[0]
        if out is None:
            out = torch.empty((B, self.out_dim), dtype=torch.float32, device=obs.device)
        s = (stream or torch.cuda.current_stream(obs.device)).cuda_stream
        self.run_device(obs.data_ptr(), out.data_ptr(), B, s)
        return out

    def run_sequence_torch(self, obs, out=None, stream=None):
        import torch
        T, B = obs.shape[0], obs.shape[1]
        if out is None:
            out = torch.empty((T, B, self.out_dim), dtype=torch.float32, device=obs.device)
        s = (stream or torch.cuda.current_stream(obs.device)).cuda_stream
        self.run_sequence_device(obs.data_ptr(), out.data_ptr(), T, B, s)
        return out

    # ------------------------------------------------------ controller tick
    def ctl_history(self):
        """kHistory of a Go2 controller policy (in_dim / 49); raises otherwise."""
        h = ctypes.c_int32()
        _check(lib().go2pi_ctl_history(self._h, ctypes.byref(h)))
        return h.value

    def ctl_set_params(self, **kw):
        """Controller parameters (go2pi_ctl_params): kp, kd, kp_stop, action_limit,
        contact_threshold, gravity_w (3), action_scale, q0 (12). Unnamed ones keep
        the reference's defaults."""
        p = CtlParams()
        lib().go2pi_ctl_default_params(ctypes.byref(p))
        for k, v in kw.items():
            if k in ("gravity_w", "q0"):
                arr = getattr(p, k)
                if len(v) != len(arr):
                    raise ValueError(f"{k} needs {len(arr)} values")
                for i, x in enumerate(v):
                    arr[i] = float(x)
            elif hasattr(p, k) and k != "struct_size":
                setattr(p, k, float(v))
            else:
                raise TypeError(f"unknown controller parameter {k!r}")
        _check(lib().go2pi_ctl_set_params(self._h, ctypes.byref(p)))

    def controller_step(self, state, obs, action, joy=None, outputs=True):
        """One controller tick on host arrays (go2pi_controller_step).
        state [B, 36] float32; joy [B, 5] float32 or None; obs [B, in_dim] and
        action [B, 12] float32 C-contiguous arrays updated IN PLACE (the
        reference's observation_ / action_). Returns (q_des, kp, kd, status) or
        None when outputs=False."""
        st = _f32(state).reshape(-1, CTL_STATE_DIM)
        B = st.shape[0]
        for name, a, w in (("obs", obs, self.in_dim), ("action", action, CTL_DOF)):
            if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous
                    and a.size == B * w):
                raise ValueError(f"{name} must be a C-contiguous float32 array of [B, {w}]")
        jy = None if joy is None else _f32(joy, B * CTL_JOY_DIM)
        res = None
        ptrs = [None, None, None, None]
        if outputs:
            res = (np.empty((B, CTL_DOF)), np.empty((B, CTL_DOF)), np.empty((B, CTL_DOF)),
                   np.empty(B, np.uint32))
            ptrs = [r.ctypes.data for r in res]
        _check(lib().go2pi_controller_step(self._h, st.ctypes.data, None if jy is None else jy.ctypes.data,
                                           obs.ctypes.data, action.ctypes.data, *ptrs, B))
        return res

    def controller_step_device(self, state_ptr, joy_ptr, obs_ptr, action_ptr, q_des_ptr, kp_ptr, kd_ptr,
                               status_ptr, batch, stream=None):
        _check(lib().go2pi_controller_step_device(self._h, state_ptr, joy_ptr, obs_ptr, action_ptr, q_des_ptr,
                                                  kp_ptr, kd_ptr, status_ptr, int(batch), stream))

    def controller_step_torch(self, state, obs, action, joy=None, q_des=None, kp=None, kd=None, status=None,
                              stream=None):
        """Device tensors: state [B,36] f32, joy [B,5] f32 or None, obs [B,in] and
        action [B,12] f32 (updated in place), optional q_des/kp/kd [B,12] float64
        and status [B] int32 outputs. Enqueued on torch's current stream (or `stream`)."""
        import torch

        def ptr(t, dtype, width):
            if t is None:
                return None
            if t.dtype != dtype or not t.is_contiguous() or t.device.type != "cuda" or t.numel() != B * width:
                raise ValueError(f"tensor must be contiguous {dtype} [B, {width}] on the GPU")
            return t.data_ptr()
        B = state.shape[0]
        args = [ptr(state, torch.float32, CTL_STATE_DIM), ptr(joy, torch.float32, CTL_JOY_DIM),
                ptr(obs, torch.float32, self.in_dim), ptr(action, torch.float32, CTL_DOF),
                ptr(q_des, torch.float64, CTL_DOF), ptr(kp, torch.float64, CTL_DOF), ptr(kd, torch.float64, CTL_DOF),
                ptr(status, torch.int32, 1)]
        s = (stream or torch.cuda.current_stream(state.device)).cuda_stream
        self.controller_step_device(*args, B, s)

    # ------------------------------------------------------ recurrent state
    def reset_hidden(self, mask=None, batch=None):
        if mask is None:
            _check(lib().go2pi_reset_hidden(self._h, None, 0))
        else:
            m = np.ascontiguousarray(mask, dtype=np.uint8)
            _check(lib().go2pi_reset_hidden(self._h, m.ctypes.data, m.size if batch is None else batch))

    def get_hidden(self, batch):
        h = np.empty((batch, self.hidden_dim), np.float32)
        _check(lib().go2pi_get_hidden(self._h, h.ctypes.data, batch))
        return h

    def set_hidden(self, h):
        h = _f32(h).reshape(-1, self.hidden_dim)
        _check(lib().go2pi_set_hidden(self._h, h.ctypes.data, h.shape[0]))

    def sync(self):
        _check(lib().go2pi_sync(self._h))

    def diag_stamps(self, n):
        """Per-workgroup {memtime, realtime} start/end stamps (diagnostic builds only)."""
        buf = np.zeros(n, np.uint64)
        k = lib().go2pi_diag_stamps(self._h, buf.ctypes.data, buf.size)
        if k < 0:
            _check(k)
        return buf[:k]

    def close(self):
        if getattr(self, "_h", None):
            lib().go2pi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def version():
    return lib().go2pi_version().decode()


def inspect_model(path):
    """The C++ loader's view of an ONNX policy (no device needed): dict."""
    import json
    cap = 1 << 16
    buf = ctypes.create_string_buffer(cap)
    n = lib().go2pi_inspect_model(os.fsencode(path), buf, cap)
    if n < 0:
        _check(n)
    if n >= cap:
        buf = ctypes.create_string_buffer(n + 1)
        lib().go2pi_inspect_model(os.fsencode(path), buf, n + 1)
    return json.loads(buf.value.decode())
