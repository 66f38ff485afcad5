"""Build libtts_hip.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

    python -m gonova_tts_amd.build          (or __graft_entry__.build())

Each csrc/*.hip / *.cpp is compiled to build/<name>.o (skipped when newer than
its sources/headers), then linked into gonova-tts_amd/libtts_hip.so which
travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libtts_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
          "-Wno-unused-result", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def _compile(src, force, build_dir=BUILD, defines=()):
    obj = os.path.join(build_dir, os.path.basename(src) + ".o")
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj, False
    cmd = [HIPCC] + CFLAGS + list(defines) + ["-x", "hip", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
    return obj, True


def build(force: bool = False, verbose: bool = True, variant: str = "", defines=(), only=()) -> str:
    """variant/defines: an A/B build (-D tunables) into build_<variant>/ and
    libtts_hip_<variant>.so, loaded with TTS_LIB=<path> (tools/ab.sh); the product is LIB.
    only: source basenames the variant recompiles (the defines touch nothing else); every other
    object comes from the product build."""
    build_dir = BUILD + ("_" + variant if variant else "")
    lib = LIB if not variant else os.path.join(PKG, f"libtts_hip_{variant}.so")
    os.makedirs(build_dir, exist_ok=True)
    srcs = _sources()
    if only and variant:
        build(verbose=False)  # the product objects the variant reuses
    mine = [s for s in srcs if not (only and variant) or os.path.basename(s) in only]
    jobs = min(len(mine), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, build_dir, defines), mine))
    objs = [o for o, _ in results] + [os.path.join(BUILD, os.path.basename(s) + ".o") for s in srcs if s not in mine]
    rebuilt = any(r for _, r in results)
    # relink when any object is newer than the library too: a variant built with `only` links the
    # product's objects, which the nested product build above may have recompiled
    stale = not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs)
    if rebuilt or stale or force:
        cmd = [HIPCC, "-shared", "-fPIC", "-Wl,-z,defs", f"--offload-arch={ARCH}", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
        if verbose:
            print(f"[gonova_tts_amd] built {lib}")
    return lib


if __name__ == "__main__":
    a = sys.argv[1:]
    var = a[a.index("--variant") + 1] if "--variant" in a else ""
    only = tuple(a[a.index("--only") + 1].split(",")) if "--only" in a else ()
    build(force="--force" in a or bool(var), variant=var, defines=[x for x in a if x.startswith("-D")], only=only)
