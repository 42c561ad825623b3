"""In-tree native build: csrc/*.hip + csrc/*.cpp -> libdmlp.so (gfx950), plus the standalone
MPI/RCCL `knn_engine` harness binary.

No torch.utils.cpp_extension (which would hipify), no JIT cache under ~/.cache: plain hipcc /
g++ invocations with an mtime check, so the .so travels with the repo snapshot to the GPU box.

    python -m distributed_machine_learning_project_amd.build [--force] [--no-engine]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = PKG / "libdmlp.so"
ENGINE = PKG / "knn_engine"
ARCH = os.environ.get("DMLP_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
MPI_HOME = os.environ.get("DMLP_MPI_HOME", "/opt/conda")

HIPCC = os.path.join(ROCM, "bin", "hipcc")
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-Wno-unused-but-set-variable"]

# screen_x1: fmaxf over MFMA results without the IEEE-mode NaN quieting (v_max_f32 x, x, x per
# operand); the kernel never produces or compares NaN
PER_FILE = {"screen_x1.hip": ["-fno-honor-nans"]}


def _sources():
    hip = sorted(CSRC.glob("*.hip"))
    cpp = sorted(p for p in CSRC.glob("*.cpp")
                 if not p.name.startswith(("engine_", "dropin_")))
    return hip, cpp


def _headers():
    return sorted(CSRC.glob("*.h"))


def _included(srcs):
    """The csrc headers these sources include, transitively (#include "x.h"): a library object
    does not go stale when only an engine-side header (engine_core.h, ...) changes."""
    import re
    seen, todo = set(), list(srcs)
    while todo:
        f = todo.pop()
        for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read_text(errors="replace"), re.M):
            h = CSRC / name
            if h.exists() and h not in seen:
                seen.add(h)
                todo.append(h)
    return sorted(seen)


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
    return r


# what the last build() did (written to _build/build_info.json and returned by build_info()):
# the driver's "build mode" — sources compiled vs objects reused, and whether the library and
# knn_engine were relinked — instead of a silent up-to-date check
_INFO = {"compiled": [], "reused": [], "lib_relinked": False, "engine_relinked": False,
         "lib_matches_sources": False, "source_hash_16": None}


def _obj_hash(src: Path) -> str:
    import hashlib
    h = hashlib.sha256(repr((ARCH, COMMON, PER_FILE.get(src.name, []))).encode())
    for f in [src] + _included([src]):
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()


def _compile(src: Path, force: bool) -> Path:
    # an object is current when the hash of its source, included headers and flags recorded
    # beside it matches (content, not mtimes: a checkout of older sources recompiles)
    obj = BUILD / (src.name + ".o")
    stamp = obj.with_name(obj.name + ".srchash")
    want = _obj_hash(src)
    if not force and obj.exists() and stamp.exists() and stamp.read_text().strip() == want:
        _INFO["reused"].append(src.name)
        return obj
    _INFO["compiled"].append(src.name)
    if src.suffix == ".hip":
        # MFMA results in VGPRs: the epilogue reads every accumulator with VALU, and AGPR
        # results cost a v_accvgpr_read per value plus copies of the C-init operand
        cmd = [HIPCC, f"--offload-arch={ARCH}", *COMMON, "-mllvm", "-amdgpu-mfma-vgpr-form=true",
               *PER_FILE.get(src.name, []), "-c", str(src), "-o", str(obj)]
    else:
        # host-only code: plain g++ without -march (no FMA contraction, SSE2 like the reference)
        cmd = ["g++", *COMMON, f"-I{CSRC}", "-pthread", "-c", str(src), "-o", str(obj)]
    _run(cmd)
    stamp.write_text(want + "\n")
    return obj


SRCHASH = LIB.with_name(LIB.name + ".srchash")  # travels with the library (untracked, like it)


def _source_hash(srcs) -> str:
    """sha256 over what the library is built from: every source and included header (name and
    bytes), the compile flags and the target — the library's identity, whatever the mtimes."""
    import hashlib
    h = hashlib.sha256(repr((ARCH, COMMON, sorted(PER_FILE.items()))).encode())
    for f in sorted(set(srcs) | set(_included(srcs))):
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()


def build_lib(force: bool = False, jobs: int | None = None) -> Path:
    BUILD.mkdir(exist_ok=True)
    hip, cpp = _sources()
    srcs = hip + cpp
    want = _source_hash(srcs)
    _INFO["source_hash_16"] = want[:16]
    force = force or os.environ.get("DMLP_BUILD_FORCE", "") == "1"
    if (not force and LIB.exists() and SRCHASH.exists() and SRCHASH.read_text().strip() == want):
        # the library was linked from exactly these sources, flags and target: up to date even
        # where its objects did not travel (a GPU box gets the tree without _build/) or the
        # mtimes moved (a checkout) — no recompile there
        _INFO["reused"].extend(s.name for s in srcs)
        _INFO["lib_matches_sources"] = True
        return LIB
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or _INFO["compiled"] or _stale(LIB, objs) or not SRCHASH.exists() or \
            SRCHASH.read_text().strip() != want:
        tmp = LIB.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp),
              "-pthread"])
        os.replace(tmp, LIB)
        _INFO["lib_relinked"] = True
    SRCHASH.write_text(want + "\n")
    _INFO["lib_matches_sources"] = True
    return LIB


def build_engine(force: bool = False) -> Path | None:
    """Standalone harness binary (MPI bootstrap + RCCL data plane + libdmlp kernels)."""
    srcs = sorted(CSRC.glob("engine_*.cpp"))
    if not srcs:
        return None
    mpi_inc = Path(MPI_HOME) / "include" / "mpi.h"
    if not mpi_inc.exists():
        print(f"[dmlp.build] no MPI headers under {MPI_HOME}; skipping knn_engine", file=sys.stderr)
        return None
    deps = srcs + _headers() + [LIB]
    if not force and not _stale(ENGINE, deps):
        return ENGINE
    BUILD.mkdir(exist_ok=True)
    objs = []
    for s in srcs:  # host-only C++ against the HIP runtime / RCCL / MPI headers
        o = BUILD / (s.name + ".o")
        _run(["g++", "-O3", "-std=c++17", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__",
              "-Werror=return-type", f"-I{CSRC}", f"-I{MPI_HOME}/include", f"-I{ROCM}/include",
              "-c", str(s), "-o", str(o)])
        objs.append(str(o))
    # MPICH lives in the conda prefix next to an old libstdc++: never put that directory on the
    # link/run path (ROCm needs the system libstdc++).  Link libmpi by its own path through a
    # private symlink directory; libmpi finds its Fortran runtime through its own RUNPATH.
    mpidir = PKG / "mpi_runtime"
    mpidir.mkdir(exist_ok=True)
    for name in ("libmpi.so.12", "libgfortran.so.4", "libquadmath.so.0"):
        src = Path(MPI_HOME) / "lib" / name
        dst = mpidir / name
        if src.exists() and not dst.is_symlink():
            dst.symlink_to(src)
    link = mpidir / "libmpi.so.12"
    _run(["g++", *objs, "-o", str(ENGINE), f"-L{PKG}", "-ldmlp", "-Wl,-rpath,$ORIGIN",
          str(link), "-Wl,-rpath,$ORIGIN/mpi_runtime", f"-L{ROCM}/lib", "-lrccl", "-lamdhip64",
          f"-Wl,-rpath,{ROCM}/lib", "-pthread"])
    _INFO["engine_relinked"] = True
    return ENGINE


def _engine_link_flags():
    mpidir = PKG / "mpi_runtime"
    return [f"-L{PKG}", "-ldmlp", f"-Wl,-rpath,{PKG}", str(mpidir / "libmpi.so.12"),
            f"-Wl,-rpath,{mpidir}", f"-L{ROCM}/lib", "-lrccl", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib",
            "-pthread"]


def build_dropin(common_cpp: str, out: str | None = None, debug: bool = False,
                 extra_flags=(), inplace: bool = False) -> Path:
    """Link the reference's own harness (its unmodified common.cpp and common.h) with
    include/engine.h + dropin_engine.cpp into a reference-compatible `engine` binary
    (Makefile:10-15 equivalent; debug=True is the engine.debug target).

    common.cpp includes "engine.h" from its own directory (common.cpp:8), so it is compiled from
    a private staging directory holding copies of common.cpp / common.h next to this package's
    engine.h — never against a sibling engine.h in the reference tree.  (dropin_engine.cpp keeps
    no state in the Engine object, so a binary built against the reference's engine.h works
    too: inplace=True compiles common.cpp where it is, against whatever engine.h sits next to it,
    exactly like the reference's Makefile with dropin_engine.cpp in place of engine.cpp.)"""
    import tempfile
    build(engine=True)  # libdmlp + the MPI runtime links
    common_cpp = Path(common_cpp).resolve()
    # default output in this package's build directory (never written into the harness's tree)
    BUILD.mkdir(exist_ok=True)
    out = Path(out or (BUILD / ("engine.debug" if debug else "engine"))).resolve()
    # up to date: same flags (a stamp beside the binary) and newer than its inputs
    stamp = out.with_name(out.name + ".flags")
    key = repr((str(common_cpp), debug, list(extra_flags), inplace))
    deps = [common_cpp, CSRC / "dropin_engine.cpp", PKG / "include" / "engine.h", LIB] + _headers()
    hdr0 = common_cpp.parent / "common.h"
    if hdr0.exists():
        deps.append(hdr0)
    if (stamp.exists() and stamp.read_text() == key and not _stale(out, deps)):
        return out
    with tempfile.TemporaryDirectory(dir=BUILD, prefix="dropin_") as td:
        stage = Path(td)
        if inplace:
            src, inc = common_cpp, common_cpp.parent
        else:
            src, inc = stage / "common.cpp", stage
            shutil.copyfile(common_cpp, src)
            hdr = common_cpp.parent / "common.h"
            if hdr.exists():
                shutil.copyfile(hdr, stage / "common.h")
            shutil.copyfile(PKG / "include" / "engine.h", stage / "engine.h")
        flags = ["-O3", "-std=c++17", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__",
                 f"-I{inc}", f"-I{CSRC}", f"-I{common_cpp.parent}", f"-I{MPI_HOME}/include",
                 f"-I{ROCM}/include", *extra_flags]
        if debug:
            flags += ["-g", "-DDEBUG"]
        _run(["g++", *flags, str(src), str(CSRC / "dropin_engine.cpp"), "-o", str(out),
              *_engine_link_flags()])
    stamp.write_text(key)
    return out


REF_HARNESS = Path(os.environ.get("DMLP_REF_HARNESS", "/root/reference"))
REF_STAGE = PKG / "_refharness"  # git-ignored, NOT gpurun-ignored (unlike _build/)


def reference_harness() -> Path | None:
    """The reference's common.cpp to build the drop-in against: the reference tree when this
    machine has it, else the untracked copy build() staged in _refharness (it travels with
    the working tree to GPU boxes, which have no reference tree; it is never committed)."""
    for d in (REF_HARNESS, REF_STAGE):
        if (d / "common.cpp").exists() and (d / "common.h").exists():
            return d / "common.cpp"
    return None


def stage_reference_harness() -> Path | None:
    """Copy the reference harness files (common.cpp, common.h, engine.h) into _refharness
    (git-ignored) so drop-in tests and `bench.py --harness dropin` can build against the
    reference's unmodified harness on a machine without the reference tree."""
    if not (REF_HARNESS / "common.cpp").exists():
        return None
    REF_STAGE.mkdir(parents=True, exist_ok=True)
    for f in ("common.cpp", "common.h", "engine.h"):
        if (REF_HARNESS / f).exists():
            # copy + atomic rename: concurrent builders (pytest -n workers) never see a
            # half-written or missing file
            tmp = REF_STAGE / f"{f}.{os.getpid()}.tmp"
            shutil.copyfile(REF_HARNESS / f, tmp)
            os.replace(tmp, REF_STAGE / f)
    return REF_STAGE / "common.cpp"


def build(force: bool = False, engine: bool = True) -> Path:
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    import time
    t0 = time.time()
    for key in ("compiled", "reused"):
        _INFO[key] = []
    _INFO["lib_relinked"] = _INFO["engine_relinked"] = False
    _INFO["lib_matches_sources"] = False
    lib = build_lib(force)
    if engine:
        build_engine(force)
    stage_reference_harness()
    _write_info(time.time() - t0)
    return lib


def _write_info(seconds: float):
    import hashlib
    import json
    info = dict(_INFO, arch=ARCH, seconds=round(seconds, 2),
                mode="rebuilt" if _INFO["compiled"] or _INFO["lib_relinked"] else "up-to-date",
                lib_sha256_16=hashlib.sha256(LIB.read_bytes()).hexdigest()[:16] if LIB.exists()
                else None)
    BUILD.mkdir(exist_ok=True)
    (BUILD / "build_info.json").write_text(json.dumps(info, indent=1) + "\n")
    print(f"[dmlp.build] {info['mode']}: {len(info['compiled'])} sources compiled, "
          f"{len(info['reused'])} objects reused, libdmlp.so relinked: {info['lib_relinked']}, "
          f"knn_engine relinked: {info['engine_relinked']} ({info['seconds']} s, {ARCH}, "
          f"libdmlp {info['lib_sha256_16']})", file=sys.stderr)


def build_info() -> dict:
    """What the last build() in this process did (see _write_info)."""
    return dict(_INFO)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-engine", action="store_true")
    ap.add_argument("--dropin", metavar="COMMON_CPP",
                    help="build a reference-compatible engine from the reference's common.cpp")
    ap.add_argument("--dropin-out", default=None)
    ap.add_argument("--dropin-debug", action="store_true", help="engine.debug (-DDEBUG)")
    ap.add_argument("--dropin-inplace", action="store_true",
                    help="compile common.cpp against the engine.h next to it (the reference's "
                         "own header), as its Makefile would")
    a = ap.parse_args(argv)
    p = build(force=a.force, engine=not a.no_engine)
    print(f"built {p}")
    if a.dropin:
        print(f"built {build_dropin(a.dropin, a.dropin_out, a.dropin_debug, inplace=a.dropin_inplace)}")


if __name__ == "__main__":
    main()
