"""Build and load libfwsim.so -- the gfx950 kernels behind the C ABI of include/fwsim.h.

The library is built in-tree (``tum_adlr_deep_reinforcement_learning_amd/lib/libfwsim.so``)
with hipcc for ``--offload-arch=gfx950``.  There is no CPU fallback: if the
library is missing the product path raises.
"""
import contextlib
import ctypes
import fcntl
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libfwsim.so")
HEADER = os.path.join(ROOT, "include", "fwsim.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "fwrollout.h")]
UNITS = [os.path.join(CSRC, "fw_kernels.hip"), os.path.join(CSRC, "fw_rollout.hip")]
SOURCES = UNITS + [os.path.join(CSRC, "fw_device.hpp"), os.path.join(CSRC, "fw_quad.hpp"), os.path.join(CSRC, "fw_stats.hpp"), os.path.join(CSRC, "fw_x8_consts.inc")] + HEADERS
ARCH = os.environ.get("FWSIM_ARCH", "gfx950")

_lib = None
ABI_VERSION = 12  # include/fwsim.h FWSIM_ABI_VERSION


class FwError(RuntimeError):
    pass


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def needs_build():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(s) > t for s in SOURCES if os.path.exists(s))


EXTRA_FLAGS = ["-fno-slp-vectorize"]  # packed-f32 pairing costs register moves here


@contextlib.contextmanager
def _build_lock(out):
    """Exclusive lock next to the library: concurrent ranks (torchrun) build once, the others wait."""
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out + ".lock", "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


N_PARTS = 7  # fw_kernels.hip build parts (FW_PART 0..6, see the file's header)


def _jobs():
    try:
        return max(1, int(os.environ.get("MAX_JOBS", "")))
    except ValueError:
        return max(1, min(8, os.cpu_count() or 1))


def build(force=False, verbose=False, out=None, extra=None):
    """Compile csrc/*.hip into lib/libfwsim.so (cross-compiles without a GPU).

    fw_kernels.hip is compiled as N_PARTS translation units in parallel (the step kernels' template
    instances dominate the compile time), then linked with fw_rollout.hip.  Holds a file lock around
    the staleness check and the compile, and writes through per-process temporary files, so parallel
    callers never see a partial library."""
    out = out or LIB_PATH
    with _build_lock(out):
        if out == LIB_PATH and not force and not needs_build():
            return LIB_PATH
        tag = "%d" % os.getpid()
        tmp = "%s.%s.tmp" % (out, tag)
        flags = EXTRA_FLAGS if extra is None else extra
        base = [_hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC"] + flags
        units = [(UNITS[0], ["-DFW_PART=%d" % p]) for p in range(N_PARTS)] + [(u, []) for u in UNITS[1:]]
        objs = ["%s.%s.%d.o" % (out, tag, k) for k in range(len(units))]
        cmds = [base + d + ["-c", "-o", o, src] for (src, d), o in zip(units, objs)]
        try:
            pending, running = list(cmds), []
            while pending or running:
                while pending and len(running) < _jobs():
                    c = pending.pop(0)
                    if verbose:
                        print(" ".join(c))
                    running.append((subprocess.Popen(c), c))
                p, c = running.pop(0)
                if p.wait() != 0:
                    for q, _ in running:
                        q.wait()
                    raise subprocess.CalledProcessError(p.returncode, c)
            link = [_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
            if verbose:
                print(" ".join(link))
            subprocess.check_call(link)
            os.replace(tmp, out)
        finally:
            for f in objs + [tmp]:
                if os.path.exists(f):
                    os.remove(f)
    return out


_c = ctypes
_vp = _c.c_void_p
_i32 = _c.c_int32
_i64 = _c.c_int64

# name -> (restype, argtypes); must match include/fwsim.h
SIGNATURES = {
    "fw_abi_version": (_c.c_int, []),
    "fw_last_error": (_c.c_int, [_c.c_char_p, _c.c_size_t]),
    "fw_create": (_c.c_int, [_vp, _vp, _i64, _i32, _i32, _c.POINTER(_vp)]),
    "fw_destroy": (_c.c_int, [_vp]),
    "fw_num_envs": (_c.c_int, [_vp, _c.POINTER(_i64)]),
    "fw_num_obs": (_c.c_int, [_vp, _c.POINTER(_i32)]),
    "fw_seed": (_c.c_int, [_vp, _c.c_uint64, _i64]),
    "fw_set_noise": (_c.c_int, [_vp, _vp, _i64]),
    "fw_set_noise_lengths": (_c.c_int, [_vp, _vp]),
    "fw_set_env_draws": (_c.c_int, [_vp, _vp, _i32]),
    "fw_quad_auto_max": (_i64, []),
    "fw_reset": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "fw_sim_step": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fw_env_step": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "fw_env_rollout": (_c.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "fw_set_lanes": (_c.c_int, [_vp, _i32]),
    "fw_get_lanes": (_c.c_int, [_vp, _c.POINTER(_i32)]),
    "fw_observe": (_c.c_int, [_vp, _vp, _vp]),
    "fw_get_state": (_c.c_int, [_vp, _i32, _vp, _vp]),
    "fw_set_state": (_c.c_int, [_vp, _i32, _vp, _vp]),
    "fw_block_rows": (_c.c_int, [_vp, _i32, _c.POINTER(_i32)]),
    "fw_update_config": (_c.c_int, [_vp, _vp, _vp]),
    "fw_set_metrics_output": (_c.c_int, [_vp, _vp]),
    "fw_set_collect_epilogue": (_c.c_int, [_vp, _vp]),
    "fw_collect_records": (_c.c_int, [_vp, _c.POINTER(_i64), _c.POINTER(_i64)]),
    "fw_collect_pending": (_c.c_int, [_vp, _vp]),
    # include/fwrollout.h
    "fw_gae": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _c.c_double, _c.c_double, _vp, _vp, _vp]),
    "fw_moments_workspace_bytes": (_c.c_size_t, [_i64, _i32]),
    "fw_moments": (_c.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _c.c_double, _vp, _vp, _vp]),
    "fw_rms_update": (_c.c_int, [_vp, _i32, _i32, _i32, _vp, _i32, _i32, _vp]),
    "fw_vecnorm_apply": (_c.c_int, [_vp, _i64, _i32, _i64, _vp, _c.c_double, _i32, _c.c_double, _vp, _i64, _vp, _i32,
                                    _c.c_double, _vp, _vp, _vp, _vp]),
    "fw_replay_add": (_c.c_int, [_vp, _i32, _vp]),
    "fw_rollout_store": (_c.c_int, [_vp, _i32, _vp, _i32, _vp]),
    "fw_policy_forward": (_c.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fw_moments_merge": (_c.c_int, [_vp, _i32, _i32, _vp, _vp]),
    "fw_vecnorm_merge_update": (_c.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "fw_collect_policy": (_c.c_int, [_vp, _vp, _vp]),
    "fw_vecnorm_pending_update": (_c.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp]),
}


class FwCopySeg(ctypes.Structure):  # include/fwrollout.h fw_copy_seg
    _fields_ = [("src", _vp), ("dst", _vp), ("bytes", _i64)]


class FwRowSeg(ctypes.Structure):  # include/fwrollout.h fw_row_seg
    _fields_ = [("src", _vp), ("dst", _vp), ("bytes", _i64), ("stride", _i64), ("row_off", _i32), ("pad", _i32)]


class FwMlpPolicy(ctypes.Structure):  # include/fwrollout.h fw_mlp_policy
    _fields_ = [(k, _vp) for k in ("pi_w0", "pi_b0", "pi_w1", "pi_b1", "act_w", "act_b", "vf_w0", "vf_b0", "vf_w1",
                                   "vf_b1", "val_w", "val_b", "log_std", "noise_row")] + \
               [("d", _i32), ("hidden", _i32), ("act_dim", _i32), ("pad", _i32)]


class FwCollectEpilogue(ctypes.Structure):  # include/fwsim.h fw_collect_epilogue
    _fields_ = [("ret", _vp), ("gamma", _c.c_double), ("records", _vp), ("row_ctrl", _vp), ("merged", _vp),
                ("rms", _vp), ("defer", _i32), ("pad", _i32)]


class FwCollectPend(ctypes.Structure):  # include/fwsim.h fw_collect_pend (ABI 12)
    _fields_ = [("records", _vp), ("stride", _i64), ("count", _i32), ("D", _i32), ("rms_prev", _vp)]


class FwCollectIO(ctypes.Structure):  # include/fwrollout.h fw_collect_io
    _fields_ = [("obs", _vp), ("reward", _vp), ("done", _vp), ("rms", _vp), ("epsilon", _c.c_double),
                ("clip_obs", _c.c_double), ("clip_reward", _c.c_double), ("norm_obs", _i32), ("norm_reward", _i32),
                ("noise", _vp), ("low", _vp), ("high", _vp), ("clipped", _vp), ("ctrl", _vp), ("obs_rows", _vp),
                ("act_rows", _vp), ("val_rows", _vp), ("logp_rows", _vp), ("rew_rows", _vp), ("start_rows", _vp),
                ("n", _i64), ("pend", _vp), ("pend_stride", _i64), ("pend_cnt", _i32), ("has_ret", _i32),
                ("merged", _vp), ("rms_prev", _vp)]


def load(path=None):
    """Load libfwsim.so (building it first only if the sources are newer and hipcc exists).

    ``FWSIM_LIB`` may point at an alternative build (A/B experiments)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("FWSIM_LIB") or LIB_PATH
    if path == LIB_PATH and needs_build() and os.path.exists(_hipcc()):
        build()
    if not os.path.exists(path):
        raise FwError("libfwsim.so not found at %s -- run __graft_entry__.build() (no CPU fallback exists)" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.fw_abi_version() != ABI_VERSION:
        raise FwError("libfwsim ABI version mismatch")
    _lib = lib
    return lib


def last_error():
    buf = ctypes.create_string_buffer(1024)
    load().fw_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc, what=""):
    if rc != 0:
        raise FwError("%s failed (%d): %s" % (what, rc, last_error()))
    return rc
