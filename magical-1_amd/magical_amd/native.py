"""ctypes binding of the C ABI (include/magical_sim.h).

The HIP library is the only compute path: if libmagical_sim.so is missing this
module raises at import time -- there is no CPU fallback.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmagical_sim_prof.so" if os.environ.get("MAGICAL_AMD_PROFILE") == "1"
                        else "libmagical_sim.so")
if os.environ.get("MAGICAL_AMD_EXP_LIB"):   # A/B kernel experiments (tools/gpu_ab.sh): an in-tree build variant
    LIB_PATH = os.path.join(HERE, "libmagical_sim_%s.so" % os.path.basename(os.environ["MAGICAL_AMD_EXP_LIB"]))

EXPORTS = ["mg_create", "mg_bind_outputs", "mg_reset", "mg_step", "mg_render_full", "mg_get_bodies", "mg_get_arbiters",
           "mg_set_body_pose", "mg_get_errors", "mg_seed", "mg_random_actions", "mg_num_envs", "mg_step_form", "mg_enable_timing", "mg_read_timing",
           "mg_set_episode_steps", "mg_selftest_sincos", "mg_replay_lores", "mg_restack", "mg_restack_window", "mg_bind_window",
           "mg_window_start", "mg_destroy", "mg_last_error"]


class mg_config(ctypes.Structure):
    _fields_ = [("task", ctypes.c_int32), ("rand_flags", ctypes.c_int32), ("preproc", ctypes.c_int32),
                ("num_envs", ctypes.c_int32), ("device", ctypes.c_int32), ("max_episode_steps", ctypes.c_int32),
                ("base_seed", ctypes.c_uint32), ("auto_reset", ctypes.c_int32),
                ("seeds", ctypes.POINTER(ctypes.c_uint32)), ("library", ctypes.c_void_p),
                ("library_size", ctypes.c_int64)]


class mg_buffers(ctypes.Structure):
    _fields_ = [("obs_allo", ctypes.c_void_p), ("obs_ego", ctypes.c_void_p), ("obs_past", ctypes.c_void_p),
                ("reward", ctypes.c_void_p), ("done", ctypes.c_void_p), ("eval_score", ctypes.c_void_p),
                ("target", ctypes.c_void_p), ("frames_only", ctypes.c_int32)]


class NativeError(RuntimeError):
    pass


_lib = None


def load():
    """Load the in-tree HIP library (loud failure if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} not found: build it with `python -m magical_amd.build` "
                          "(no CPU fallback exists for the simulator)")
    if os.path.basename(LIB_PATH) != "libmagical_sim.so":
        # a profiling / experiment variant (MAGICAL_AMD_PROFILE, MAGICAL_AMD_EXP_LIB) is built by hand: refuse one
        # older than the sources, so no profile is taken on a stale build
        csrc = os.path.join(os.path.dirname(HERE), "csrc")
        newest = max(os.path.getmtime(os.path.join(csrc, f)) for f in os.listdir(csrc))
        if os.path.getmtime(LIB_PATH) < newest:
            raise NativeError(f"{LIB_PATH} is older than magical-1_amd/csrc: rebuild it (python -m magical_amd.build "
                              "--profile, or tools/build_unit_variant.sh) before profiling with it")
    lib = ctypes.CDLL(LIB_PATH)
    vp, i32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64
    lib.mg_create.argtypes = [ctypes.POINTER(mg_config), ctypes.POINTER(vp)]
    lib.mg_bind_outputs.argtypes = [vp, ctypes.POINTER(mg_buffers)]
    lib.mg_reset.argtypes = [vp, vp, vp]
    lib.mg_step.argtypes = [vp, vp, vp]
    lib.mg_render_full.argtypes = [vp, vp, vp]
    lib.mg_get_bodies.argtypes = [vp, vp, vp, vp]
    lib.mg_get_errors.argtypes = [vp, vp, vp]
    if hasattr(lib, "mg_get_arbiters"):
        lib.mg_get_arbiters.argtypes = [vp, vp, vp, vp]
    lib.mg_set_body_pose.argtypes = [vp, i32, i32, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
    lib.mg_seed.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32)]
    lib.mg_random_actions.argtypes = [vp, vp, u64, u64, vp]
    lib.mg_num_envs.argtypes = [vp]
    if hasattr(lib, "mg_step_form"):
        lib.mg_step_form.argtypes = [vp, vp]
    lib.mg_selftest_sincos.argtypes = [vp, vp, vp, i32, vp]
    lib.mg_enable_timing.argtypes = [vp, i32]
    lib.mg_read_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    lib.mg_set_episode_steps.argtypes = [vp, vp, vp]
    if hasattr(lib, "mg_replay_lores"):   # (a profiling build may predate it; the product library is checked
        lib.mg_replay_lores.argtypes = [vp, i32, vp, i32, vp, vp, vp, vp, vp]   # by tests/test_host.py)
    if hasattr(lib, "mg_restack"):
        i64 = ctypes.c_int64
        lib.mg_restack.argtypes = [vp, i32, i32, i64, i64, i64, i64, i32, i64, i32, vp, vp, vp, vp, vp]
    if hasattr(lib, "mg_restack_window"):
        i64 = ctypes.c_int64
        lib.mg_restack_window.argtypes = [vp, i32, i32, i64, i64, i64, i64, i32, i64, i32, i32, vp, vp]
    if hasattr(lib, "mg_bind_window"):
        lib.mg_bind_window.argtypes = [vp, vp, vp, i32]
        lib.mg_window_start.argtypes = [vp, ctypes.POINTER(i32)]
    lib.mg_destroy.argtypes = [vp]
    lib.mg_destroy.restype = None
    lib.mg_last_error.restype = ctypes.c_char_p
    for name in EXPORTS[:-2]:
        if not hasattr(lib, name):
            continue
        if getattr(lib, name).restype is ctypes.c_int:  # default
            getattr(lib, name).restype = i32
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = _lib.mg_last_error().decode() if _lib is not None else ""
        raise NativeError(f"magical_sim error {rc}: {msg}")
    return rc
