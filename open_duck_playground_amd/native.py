"""Loader for the MI355X C-ABI library (``libduck.so``, ``include/duck.h``).

The product path only ever calls into this library; there is no CPU fallback. If the
shared object is missing or fails to load, every entry point raises.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

from .cabi import DuckEnvConfig, DuckModelDesc, DuckRefMotion

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DUCK_LIB") or os.path.join(HERE, "libduck.so")
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)

BUILD = os.path.join(HERE, "build")  # libraries compiled for other models (model_library)

EXPORTS = ["duck_version", "duck_build_id", "duck_last_error", "duck_layout_get", "duck_aux_size", "duck_create", "duck_destroy",
           "duck_debug_stage_cycles", "duck_model_fingerprint", "duck_model_supported",
           "duck_reset", "duck_step", "duck_randomize", "duck_physics_step", "duck_gae", "duck_ppo_loss",
           "duck_ppo_loss_out_size", "duck_mlp_gemm", "duck_mlp_wgrad", "duck_mlp_wgrad_reduce",
           "duck_policy_sample", "duck_clip_adam", "duck_clip_adam_scratch_size", "duck_set_step_mode",
           "duck_step_kernel_for", "duck_debug_lat_timeouts", "duck_gather_columns", "duck_mlp_group",
           "duck_device_error", "duck_gae_stats", "duck_ppo_loss_stats", "duck_mlp_group_bn", "duck_gather_columns_norm",
           "duck_column_stats", "duck_column_stats_scratch", "duck_clip_adam_reduce", "duck_ppo_loss_grad",
           "duck_ppo_loss_sums", "duck_mlp_group_tiles"]


class DuckMlpProblem(C.Structure):
    """include/duck_ppo.h duck_mlp_problem"""
    _fields_ = [("kind", C.c_int), ("N", C.c_int), ("R", C.c_int), ("M", C.c_int),
                ("A", C.c_void_p), ("W", C.c_void_p), ("bias", C.c_void_p), ("aux", C.c_void_p),
                ("Y", C.c_void_p), ("Y2", C.c_void_p), ("mean", C.c_void_p), ("istd", C.c_void_p),
                ("splits", C.c_int), ("P", C.c_int), ("off_w", C.c_int), ("off_b", C.c_int), ("partial", C.c_void_p)]


class DuckGatherField(C.Structure):
    """include/duck_ppo.h duck_gather_field"""
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("T", C.c_int), ("B", C.c_int), ("w", C.c_int)]


class DuckError(RuntimeError):
    pass


class DuckLayout(C.Structure):
    _fields_ = [(k, C.c_int) for k in (
        "nq", "nv", "nu", "imitation", "task", "obs_size", "priv_size",
        "qpos", "qvel", "qacc_warmstart", "ctrl", "command", "last_act", "last_last_act", "last_last_last_act",
        "motor_targets", "feet_air_time", "last_contact", "swing_peak", "push", "action_history", "imu_history",
        "ref_motion", "imitation_phase", "metrics", "reward", "done", "truncation", "first_qpos", "first_qvel",
        "first_qacc_warmstart", "first_ctrl", "first_obs", "first_priv", "nfloat",
        "rng_key", "rng_ctr", "step", "push_step", "push_interval", "imitation_i", "ep_steps", "nint")]


# the machine scheduler's max-ILP strategy: the step kernel runs one wave per SIMD, so
# occupancy-driven scheduling buys nothing and latency hiding must come from the wave's own
# instruction stream (same-box A/B: +3 % env-steps/s). Every unit uses it; the build is
# gated by tools/isa_exec_check.py, which rejects the register-allocation fault that once made
# the rough + backlash physics_kernel compute a wrong Newton step.
ILP_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]


def _base_flags(inc: str) -> list:
    # fp32 division and sqrt as v_rcp/v_sqrt (1-2 ulp) instead of the correctly rounded
    # multi-instruction sequences: the physics tolerances are fp32-vs-fp64 anyway; fp32
    # denormals flushed (no frexp/ldexp range scaling around v_rcp/v_sqrt/sincos); x/y as
    # x*rcp(y) and signed zeros ignored (+0.8 % same-box, parity unchanged) -- NaN/Inf stay
    # honoured: the termination check and the auto-reset NaN guard depend on them
    return ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-hip-fp32-correctly-rounded-divide-sqrt",
            "-fgpu-flush-denormals-to-zero", "-fno-slp-vectorize",
            "-fno-signed-zeros", "-fno-trapping-math", "-fno-math-errno", "-freciprocal-math", "-I" + CSRC,
            "-I" + inc]


def compile_flags() -> list:
    """The hipcc flags of the shipped scene units (tools: occupancy_probe.sh, ISA studies)."""
    return _base_flags(os.path.join(CSRC, "generated")) + ILP_FLAGS


def build(verbose: bool = False, defines=(), out: str = None, extra_flags=(), no_ilp=(), isa_check: bool = True,
          gen_dir: str = None) -> str:
    """Compile libduck.so for gfx950 with hipcc (in-tree, so it travels with the repo).

    One translation unit per model variant (variant_*.hip) plus the C ABI (duck_capi.hip),
    compiled in parallel and linked into one shared library. ``gen_dir`` (model_library) holds
    the units, headers and variant registry of other models instead of the four shipped scenes.
    One builder per output at a time (torchrun ranks importing the package together): the others
    wait on a file lock and then find the library fresh, so N ranks run one hipcc build, not N."""
    import fcntl
    out = os.path.abspath(out or LIB_PATH)
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, os.path.basename(out) + ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            # the freshness check runs under the lock: a rank never scans a library another rank
            # is still replacing
            return _build_unlocked(verbose, defines, out, extra_flags, no_ilp, isa_check, gen_dir)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)


def _build_unlocked(verbose, defines, out, extra_flags, no_ilp, isa_check, gen_dir) -> str:
    if gen_dir is None:
        srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
        inc = os.path.join(CSRC, "generated")
    else:
        srcs = [os.path.join(CSRC, "duck_capi.hip")] + \
            sorted(os.path.join(gen_dir, f) for f in os.listdir(gen_dir) if f.endswith(".hip"))
        inc = gen_dir
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(inc, f) for f in os.listdir(inc)] + \
        [os.path.join(ROOT, "include", f) for f in sorted(os.listdir(os.path.join(ROOT, "include"))) if f.endswith(".h")] + \
        [os.path.abspath(__file__)]  # the compile flags live here
    # (a define/flag build into the shared output is never "fresh"; a unit directory's own output is)
    if (gen_dir is not None or not defines and not extra_flags) and os.path.exists(out) and \
            os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    import hashlib
    import tempfile
    flags = _base_flags(inc) + [f"-D{d}" for d in defines] + list(extra_flags)
    ilp = ILP_FLAGS
    # build id: sha1 of every source, header and flag that shapes the code (duck_build_id()); the
    # .so itself is not byte-reproducible (object paths), so profiles are keyed by this instead
    h = hashlib.sha1(" ".join(flags + ilp + sorted(no_ilp)).encode())
    for d in sorted(set(deps) - {os.path.abspath(__file__)}):
        h.update(os.path.relpath(d, ROOT).encode())
        h.update(open(d, "rb").read())
    flags = flags + [f'-DDUCK_BUILD_ID="{h.hexdigest()}"']
    with tempfile.TemporaryDirectory() as tmp:
        objs, procs = [], []
        for src in srcs:
            obj = os.path.join(tmp, os.path.basename(src) + ".o")
            cmd = ["hipcc"] + flags + ([] if os.path.basename(src) in no_ilp else ilp) + ["-c", "-o", obj, src]
            if verbose:
                print(" ".join(cmd))
            procs.append((src, subprocess.Popen(cmd, cwd=CSRC)))
            objs.append(obj)
        bad = [src for src, p in procs if p.wait() != 0]
        if bad:
            raise DuckError(f"hipcc failed on {bad}")
        # a per-process temporary: concurrent builders (ranks, model_library callers) never link over
        # or scan each other's file; os.replace publishes the checked library atomically
        tmp_out = f"{out}.{os.getpid()}.tmp"
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-o", tmp_out] + objs, cwd=CSRC)
    try:
        if isa_check:
            nvar = sum(os.path.basename(f).startswith("variant_") for f in srcs)
            bad = isa_exec_faults(tmp_out, min_step_kernels=nvar)
            if bad:
                raise DuckError("register-allocation fault in the compiled kernels (split copies ahead of an exec "
                                "restore, tools/isa_exec_check.py):\n" + "\n".join(bad))
        os.replace(tmp_out, out)
    finally:
        if os.path.exists(tmp_out):
            os.remove(tmp_out)
    return out


def model_library(m, verbose: bool = False) -> str:
    """The library whose kernels are compiled for model ``m``: libduck.so when ``m`` is one of the
    shipped scenes, else ``build/libduck_<fingerprint>.so``, generated and compiled on first use
    (codegen.model_header; the model compiler's structural checks apply). The MI355X analogue of
    MJX re-specialising its program when the MJCF changes: an edited XML needs no hand edits."""
    from . import codegen
    from .cabi import model_fingerprint
    fp = model_fingerprint(m)
    for var, task in codegen.DEFAULT_VARIANTS:
        hdr = os.path.join(CSRC, "generated", f"duck_model_{var}.h")
        if os.path.exists(hdr) and f"FINGERPRINT = 0x{fp:016x}ull" in open(hdr).read():
            return LIB_PATH
    import fcntl
    name = f"m{fp:016x}"
    out = os.path.join(BUILD, f"libduck_{name}.so")
    gen = os.path.join(BUILD, f"gen_{name}")
    os.makedirs(gen, exist_ok=True)
    # one builder per model at a time (torchrun ranks, several envs on the same edited XML): the
    # others wait on the lock and then find the library fresh
    with open(os.path.join(BUILD, f"libduck_{name}.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            # regenerate first: a codegen change that alters the header or unit rewrites it, and
            # build()'s freshness check (sources, headers, include/, native.py) then rebuilds
            files = {f"duck_model_{name}.h": codegen.model_header(m, name),
                     f"variant_{name}.hip": codegen.variant_unit(name, f"duck_model_{name}.h"),
                     "duck_variants.inc": codegen.variant_registry([name])}
            for fn, text in files.items():
                path = os.path.join(gen, fn)
                if not os.path.exists(path) or open(path).read() != text:
                    with open(path, "w") as f:
                        f.write(text)
            return build(verbose=verbose, out=out, gen_dir=gen)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)


def debug_library(name: str, defines, variants=("flat",), verbose: bool = False) -> str:
    """build/libduck_<name>.so: the shipped scene variants in `variants` compiled with extra `defines`
    (test builds, e.g. DUCK_LAT_FORCE_TIMEOUT for test_gpu_env.py::test_latency_timeout_surfaces).
    One scene instead of four keeps the build short; built by __graft_entry__.build(), never on a GPU box."""
    from . import codegen
    gen = os.path.join(BUILD, f"gen_{name}")
    os.makedirs(gen, exist_ok=True)
    # (the defines are a file of the unit directory: a change of them makes build() recompile)
    files = {"duck_variants.inc": codegen.variant_registry(variants), "defines.txt": "\n".join(defines) + "\n"}
    for v in variants:
        files[f"duck_model_{v}.h"] = open(os.path.join(CSRC, "generated", f"duck_model_{v}.h")).read()
        files[f"variant_{v}.hip"] = codegen.variant_unit(v, f"duck_model_{v}.h")
    for fn, text in files.items():
        path = os.path.join(gen, fn)
        if not os.path.exists(path) or open(path).read() != text:
            with open(path, "w") as f:
                f.write(text)
    return build(verbose=verbose, defines=tuple(defines), out=os.path.join(BUILD, f"libduck_{name}.so"), gen_dir=gen)


def isa_kernels(texts) -> list:
    """The kernel symbols (amdgpu_kernel entry labels) in disassembled code objects."""
    import re
    out = []
    for t in texts:
        out += re.findall(r"^[0-9a-f]+ <(_Z\d+(?:step|physics|reset|randomize)_kernel\w*)>:$", t, re.M)
    return out


def isa_exec_faults(so_path: str, min_step_kernels: int = 1):
    """Blocks of the gfx950 code in so_path whose exec-restoring join starts with AGPR/scratch moves
    (tools/isa_exec_check.py): each is a lane-masked live-range split, i.e. a wrong-result kernel.
    Fails closed: raises DuckError when no code object could be disassembled or fewer than
    min_step_kernels step_kernel / physics_kernel symbols were scanned (a missing fat binary, an
    unbundling failure or a compressed bundle must not pass as "no faults")."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_exec_check", os.path.join(ROOT, "tools", "isa_exec_check.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    texts = mod.code_objects(so_path)
    kern = isa_kernels(texts)
    nstep = sum("step_kernel" in k for k in kern)
    nphys = sum("physics_kernel" in k for k in kern)
    if not texts or nstep < min_step_kernels or nphys < min_step_kernels:
        raise DuckError(f"ISA gate scanned nothing usable in {so_path}: {len(texts)} code object(s), "
                        f"{nstep} step_kernel / {nphys} physics_kernel symbol(s), {min_step_kernels} expected")
    found = []
    for text in texts:
        found += mod.scan(text, os.path.basename(so_path))
    return [f"{func[:80]}: {len(pre)} move(s) before '{ins}'" for _, func, _, pre, ins in found]


_libs = {}


def lib(path: str = None):
    """Load libduck.so, or the library at ``path`` (raises if it is missing: no fallback path exists)."""
    path = os.path.abspath(path or LIB_PATH)
    if path not in _libs:
        if not os.path.exists(path):
            raise DuckError(f"{path} not built; run __graft_entry__.build() or native.build()")
        L = C.CDLL(path)
        vp = C.c_void_p
        L.duck_version.restype = C.c_int
        L.duck_build_id.restype = C.c_char_p
        L.duck_last_error.restype = C.c_char_p
        L.duck_layout_get.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(DuckLayout)]
        L.duck_aux_size.argtypes = [vp]
        L.duck_create.argtypes = [C.POINTER(DuckModelDesc), C.POINTER(DuckEnvConfig), C.POINTER(DuckRefMotion), C.c_int,
                                  C.POINTER(vp)]
        L.duck_destroy.argtypes = [vp]
        L.duck_destroy.restype = None
        L.duck_reset.argtypes = [vp, C.c_int, vp, vp, vp, C.c_uint64, C.c_int64, vp, vp, vp, vp]
        L.duck_step.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.duck_randomize.argtypes = [vp, C.c_int, vp, C.c_uint64, C.c_int64, vp]
        L.duck_physics_step.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp, vp, vp]
        L.duck_model_fingerprint.restype = C.c_uint64
        L.duck_model_fingerprint.argtypes = [C.POINTER(DuckModelDesc)]
        L.duck_model_supported.argtypes = [C.POINTER(DuckModelDesc)]
        if hasattr(L, "duck_set_step_mode"):  # (libraries built before the latency kernel: A/B baselines)
            L.duck_set_step_mode.argtypes = [vp, C.c_int]
            L.duck_step_kernel_for.argtypes = [vp, C.c_int]
            L.duck_debug_lat_timeouts.argtypes = [vp, C.POINTER(C.c_uint), C.c_int]
        if hasattr(L, "duck_device_error"):
            L.duck_device_error.argtypes = [vp, C.POINTER(C.c_uint), C.c_int]
        if hasattr(L, "duck_gae"):
            L.duck_gae.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, C.c_float, C.c_float, vp, vp, vp]
        if hasattr(L, "duck_gae_stats"):
            L.duck_gae_stats.argtypes = [C.c_int, C.c_int, vp, vp, vp, C.c_float, vp, vp, C.c_float, C.c_float, vp, vp,
                                         C.c_int, vp, vp]
            L.duck_ppo_loss_stats.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_float, vp,
                                              vp, vp, vp, vp]
        if hasattr(L, "duck_ppo_loss"):
            L.duck_ppo_loss.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_float, C.c_int,
                                        vp, vp, vp, vp]
            L.duck_ppo_loss_out_size.argtypes = [C.c_int]
        if hasattr(L, "duck_mlp_group"):
            L.duck_mlp_group.argtypes = [C.c_int, C.POINTER(DuckMlpProblem), vp]
        if hasattr(L, "duck_mlp_group_bn"):
            L.duck_mlp_group_bn.argtypes = [C.c_int, C.POINTER(DuckMlpProblem), C.c_int, vp]
        if hasattr(L, "duck_mlp_group_tiles"):
            L.duck_mlp_group_tiles.argtypes = [C.c_int, C.POINTER(DuckMlpProblem), C.c_int, C.c_int, vp]
        if hasattr(L, "duck_gather_columns_norm"):
            L.duck_gather_columns_norm.argtypes = [C.c_int, C.POINTER(DuckGatherField), C.POINTER(C.c_void_p), vp,
                                                   C.c_int, vp]
        if hasattr(L, "duck_clip_adam_reduce"):
            L.duck_clip_adam_reduce.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_float,
                                                C.c_float, C.c_float, C.c_float, vp]
            L.duck_ppo_loss_grad.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_float, vp,
                                             vp, vp, vp, vp]
            L.duck_ppo_loss_sums.argtypes = [C.c_int, C.c_int, C.c_float, vp, vp]
        if hasattr(L, "duck_column_stats"):
            L.duck_column_stats.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp]
            L.duck_column_stats_scratch.argtypes = [C.c_int, C.c_int]
        if hasattr(L, "duck_gather_columns"):
            L.duck_gather_columns.argtypes = [C.c_int, C.POINTER(DuckGatherField), vp, C.c_int, vp]
        if hasattr(L, "duck_mlp_gemm"):
            ci = C.c_int
            L.duck_mlp_gemm.argtypes = [ci, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp]
            L.duck_mlp_wgrad.argtypes = [ci, ci, ci, vp, vp, vp, vp, ci, vp, ci, ci, ci, vp]
            L.duck_mlp_wgrad_reduce.argtypes = [ci, ci, vp, vp, vp]
            L.duck_policy_sample.argtypes = [ci, ci, vp, C.c_uint64, vp, vp, vp, vp, vp]
            cf = C.c_float
            L.duck_clip_adam.argtypes = [ci, vp, vp, vp, vp, vp, vp, cf, cf, cf, cf, cf, vp]
            L.duck_clip_adam_scratch_size.argtypes = [ci]
        _libs[path] = L
    return _libs[path]


def check(rc: int, L=None):
    if rc != 0:
        raise DuckError(f"libduck error {rc}: {(L or lib()).duck_last_error().decode()}")
    return rc
