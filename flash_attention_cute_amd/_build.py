"""In-tree build of the gfx950 kernels and the torch binding.

Replaces the reference's JIT build (reference flash_attention/load_cpp_extention.py:11-53), which
drives nvcc through ``torch.utils.cpp_extension.load`` and, under ROCm torch, hipifies ``.cu``
files into the source tree. Here nothing is hipified: two explicit compiler invocations write
into the package directory so the artefacts travel with the repository snapshot.

  1. ``hipcc --offload-arch=gfx950``  csrc/fa_inst.hip x 16 (one object per dtype x causal x
     head-dim tile x exact-D instantiation, compiled in parallel) + csrc/fa_fwd_gfx950.hip (C-ABI
     dispatcher)  ->  lib/libfa_gfx950.so (the C-ABI library of include/fa_gfx950.h; no torch
     symbols)
  2. ``g++``  csrc/flash_attention_api.cpp  ->  _C<ext>.so  (pybind11 torch binding, linked
     against lib/libfa_gfx950.so with an $ORIGIN rpath)

Both steps are skipped when the output is newer than every input.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
INCLUDE = ROOT / "include"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = ROCM / "bin" / "hipcc"
ARCH = "gfx950"

ABI_LIB = LIBDIR / "libfa_gfx950.so"
# the same C-ABI with the debug / A-B kernel bodies compiled in (-DFA_DEBUG_VARIANTS: fa_fwd_w8,
# fa_fwd_p8, the non-pipelined w4slow body), for the GPU test sweep and A/B scripts only
DEBUG_LIB = LIBDIR / "libfa_gfx950_debug.so"
EXT_NAME = "_C"


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"{EXT_NAME}{suffix}"


def _stale(out: Path, inputs: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(p.stat().st_mtime > t for p in inputs if p.exists())


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(str(c) for c in cmd), flush=True)
    res = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"build step failed ({res.returncode}):\n{' '.join(map(str, cmd))}\n"
                           f"{res.stdout}\n{res.stderr}")


def abi_sources() -> list[Path]:
    """Every file an instantiation TU or the dispatcher can include (any header edit rebuilds)."""
    dev = [p for ext in ("*.hip", "*.hpp", "*.h", "*.inc") for p in sorted(CSRC.glob(ext))]
    return dev + sorted(INCLUDE.glob("*.h")) + [Path(__file__).resolve(), PKG / "_asm_check.py"]


# (dtype, causal, head-dim tile, exact head dim): must match FA_FOR_EACH_INSTANCE in csrc/fa_launch.h
INSTANCES = [(dt, c, d, e) for dt in ("F16", "BF16") for c in (0, 1) for d in (64, 128) for e in (0, 1)]

HIP_FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5",
             "-ffinite-math-only", "-fno-signed-zeros"]


def _jobs() -> int:
    n = os.environ.get("MAX_JOBS") or os.cpu_count() or 4
    return max(1, min(int(n), 16))


def _process_pool():
    """Worker processes for the assembly gate (a pure-Python dataflow over each instantiation, seconds each).
    Spawned, not forked: a fork taken while the compile threads' pool still holds locks left the workers
    hung (seen twice in round 6)."""
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor

    return ProcessPoolExecutor(max_workers=_jobs(), mp_context=multiprocessing.get_context("spawn"))


def build_abi(force: bool = False, verbose: bool = False, stamps: bool = False, tag: str = "",
              defines: tuple = (), flags: tuple = (), only: tuple = (), debug: bool = False,
              gate: bool = True) -> Path:
    """Compile the HIP kernels + C-ABI into lib/libfa_gfx950.so (gfx950 code objects); ``debug``:
    lib/libfa_gfx950_debug.so, the same with the debug / A-B kernel bodies (-DFA_DEBUG_VARIANTS).

    Each kernel instantiation is its own translation unit (csrc/fa_inst.hip with -D selectors), so
    the 16 device compiles run in parallel; objects go to build/ and are linked by hipcc.
    """
    from concurrent.futures import ThreadPoolExecutor

    # diagnostic builds (stamps, experiments) go to build/stamps[_<tag>]/, never over the product
    # (experiment builds without stamps: tag + defines, to build/exp_<tag>/, for scripts/ab_libs.py)
    sdir = ("stamps" if stamps else "exp") + (f"_{tag}" if tag else "")
    diag = stamps or bool(tag)
    out_lib = ROOT / "build" / sdir / "libfa_gfx950.so" if diag else DEBUG_LIB if debug else ABI_LIB
    out_lib.parent.mkdir(parents=True, exist_ok=True)
    if not force and not _stale(out_lib, abi_sources()):
        return out_lib
    if not HIPCC.exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    objdir = ROOT / "build" / (f"obj_{sdir}" if diag else "obj_debug" if debug else "obj")
    extra = ((["-DFA_STAMPS=1"] if stamps else []) + [f"-D{d}" for d in defines] + list(flags)) if diag else []
    if debug or stamps:  # (stamp builds keep the debug bodies: scripts/stamps.py can select p8; experiment
        # builds compile what the product does, so an A/B against the product library compares like code)
        extra = ["-DFA_DEBUG_VARIANTS=1"] + extra
    objdir.mkdir(parents=True, exist_ok=True)
    cmds = []  # (command, object, inputs): an object newer than its inputs, built by the same command, is kept
    objs = []
    asm_files = []
    tooling = [Path(__file__).resolve()]
    headers = [CSRC / "fa_launch.h", *sorted(INCLUDE.glob("*.h"))]
    inst_deps = [p for ext in ("*.hpp", "*.h", "*.inc") for p in sorted(CSRC.glob(ext))] + [CSRC / "fa_inst.hip"]
    for dt, c, d, e in INSTANCES:
        # one directory per instantiation: -save-temps=obj names its files after the source
        idir = objdir / f"{dt.lower()}_c{c}_d{d}_x{e}"
        idir.mkdir(parents=True, exist_ok=True)
        obj = idir / "fa_inst.o"
        objs.append(obj)
        stub = ["-DFA_INST_STUB=1"] if only and (dt, c, d, e) not in only else []
        if not stub:
            asm_files.append(idir / f"fa_inst-hip-amdgcn-amd-amdhsa-{ARCH}.s")
        cmds.append(([HIPCC, *HIP_FLAGS, *extra, *stub, f"-I{INCLUDE}", f"-I{CSRC}", f"-DFA_INST_DT={dt}",
                      f"-DFA_INST_CAUSAL={c}", f"-DFA_INST_D={d}", f"-DFA_INST_EXACT={e}", "-save-temps=obj",
                      "-Wno-inline-asm", "-c", CSRC / "fa_inst.hip", "-o", obj], obj, inst_deps + tooling))
    for src in ("fa_fwd_gfx950.hip", "fa_rope.hip"):  # C-ABI dispatcher, standalone RoPE kernel
        obj = objdir / src.replace(".hip", ".o")
        objs.append(obj)
        cmds.append(([HIPCC, *HIP_FLAGS, *extra, f"-I{INCLUDE}", f"-I{CSRC}", "-c", CSRC / src, "-o", obj], obj,
                     [CSRC / src, *headers, *tooling]))

    def compile_one(cmd, obj, deps):
        stamp = obj.with_suffix(".cmd")
        line = " ".join(map(str, cmd))
        if (not force and not _stale(obj, deps) and stamp.exists() and stamp.read_text() == line
                and (obj.name != "fa_inst.o" or next(obj.parent.glob("*.s"), None) is not None)):
            return
        _run(cmd, verbose)
        stamp.write_text(line)

    with ThreadPoolExecutor(max_workers=_jobs()) as ex:
        for f in [ex.submit(compile_one, *c) for c in cmds]:
            f.result()
    # gate: the literal-AGPR invariant of fa_fwd_w4 and no VGPR spills (_asm_check)
    from ._asm_check import check_file

    with ThreadPoolExecutor(max_workers=1) if len(asm_files) < 2 else _process_pool() as ex:
        problems = [p for ps in ex.map(check_file, asm_files) for p in ps]
    if diag:  # stamp / experiment builds: spills are reported, not fatal (the AGPR rule stays)
        for q in [q for q in problems if "vgpr_spill_count" in q or not gate]:
            print(f"warning ({sdir}): {q}", flush=True)
        # (gate=False: an experiment that reproduces a rejected build, e.g. FA_EXP_CZERO, rule R5)
        problems = [q for q in problems if "vgpr_spill_count" not in q] if gate else []
    for a in asm_files:  # keep the .s for inspection, drop the large intermediates
        for junk in a.parent.glob("fa_inst*"):
            if junk.suffix in (".bc", ".hipi", ".out", ".txt", ".hipfb") or junk.name.endswith("resolution.txt"):
                junk.unlink()
    if problems:
        raise RuntimeError("device assembly check failed (_asm_check):\n" + "\n".join(problems[:20]))
    tmp = out_lib.with_suffix(".so.tmp")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp], verbose)
    os.replace(tmp, out_lib)
    return out_lib


def build_ext(force: bool = False, verbose: bool = False) -> Path:
    """Compile the pybind11 torch binding (host-only C++, no device code)."""
    import torch
    from torch.utils import cpp_extension

    lib = build_abi(force=force, verbose=verbose)
    out = ext_path()
    src = CSRC / "flash_attention_api.cpp"
    if not force and not _stale(out, [src, INCLUDE / "fa_gfx950.h", lib]):
        return out
    incs = cpp_extension.include_paths(device_type="cuda")
    libdirs = cpp_extension.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H",
           f"-I{INCLUDE}", f"-I{sysconfig.get_paths()['include']}"]
    cmd += [f"-I{p}" for p in incs]
    cmd += [src, "-o", out.with_suffix(".tmp")]
    cmd += [f"-L{p}" for p in libdirs]
    cmd += [f"-L{LIBDIR}", "-lfa_gfx950", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_python", "-lamdhip64", "-Wl,-rpath,$ORIGIN/lib"]
    _run(cmd, verbose)
    os.replace(out.with_suffix(".tmp"), out)
    return out


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_abi(force=force, verbose=verbose)
    build_abi(force=force, verbose=verbose, debug=True)
    build_ext(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
