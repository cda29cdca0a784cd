"""Build libalipmpc.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The library is the product: there is no CPU execution path behind it.

csrc/alipmpc.hip is compiled as 9 translation units in parallel — ALIP_PART=0 (host code, C ABI, rollout
kernels), ALIP_PART=1..6 (the solve/eval kernels of one horizon N each, fp64 and fp32) and ALIP_PART=7/8 (the
lane solver of csrc/lane_solve.inc, fp64 / fp32) — and linked into one shared library.  `ALIPMPC_SINGLE_TU=1` builds it as one TU instead (slower, same code).
"""
import hashlib
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                         # mujoco-lip-mpc-simulation_amd/
REPO = os.path.dirname(ROOT)
SRC = os.path.join(ROOT, "csrc", "alipmpc.hip")
INC = os.path.join(ROOT, "csrc", "lane_solve.inc")
MATH = os.path.join(ROOT, "csrc", "fastmath.inc")
RESTO = os.path.join(ROOT, "csrc", "resto_wave.inc")
HDR = os.path.join(REPO, "include", "alipmpc.h")
LIB = os.path.join(PKG, "libalipmpc.so")
PARTS = range(0, 9)

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = ["--offload-arch=gfx950"]
FLAGS = ["-O3", "-std=c++17", "-fPIC",
         # keep MachineLICM from hoisting f64 literals / LDS addresses out of the interior-point loop
         # (it pins ~100 VGPRs across the whole solve and forces spills)
         "-mllvm", "-disable-machine-licm",
         "-Wno-unused-value"]


def build_id(extra=(), src=None):
    """16-hex id of a build: sha256 over the sources it compiles (kernel sources, the header, this file's flags)
    and the extra flags.  Compiled into the library (alipmpc_build_id) so a counter record made with one build is
    never attached to a bench line of another (tools/roofline.py, bench.py)."""
    h = hashlib.sha256()
    for p in (src or SRC, INC, MATH, RESTO, HDR):
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join([*ARCH, *FLAGS, *extra]).encode())
    return h.hexdigest()[:16]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in (SRC, INC, MATH, RESTO, HDR, __file__))


def _run(cmd, verbose):
    if verbose:
        print("[alipmpc] " + " ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)


def build(force=False, verbose=True, extra=(), out=None, src=None):
    """Build the library (out / src: output path and source of dev variants, e.g. extra=["-DALIP_STAMPS"])."""
    target = out or LIB
    src = src or SRC
    if not force and out is None and not needs_build():
        return LIB
    tmp_lib = target + ".tmp"
    extra = [*extra, f'-DALIP_BUILD_ID="{build_id(extra, src)}"']
    if os.environ.get("ALIPMPC_SINGLE_TU") == "1":
        _run([HIPCC, *ARCH, *FLAGS, *extra, "-shared", "-o", tmp_lib, src], verbose)
    else:
        jobs = max(1, min(len(PARTS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
        with tempfile.TemporaryDirectory(prefix="alipmpc_build_") as td:
            objs = [os.path.join(td, f"part{k}.o") for k in PARTS]
            cmds = [[HIPCC, *ARCH, *FLAGS, *extra, f"-DALIP_PART={k}", "-c", "-o", o, src]
                    for k, o in zip(PARTS, objs)]
            with ThreadPoolExecutor(jobs) as ex:
                for f in [ex.submit(_run, c, verbose) for c in cmds]:
                    f.result()
            _run([HIPCC, *ARCH, "-shared", "-fPIC", "-o", tmp_lib, *objs], verbose)
    os.replace(tmp_lib, target)
    return target


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", default=None, help="dev variant output path")
    ap.add_argument("-D", dest="defs", action="append", default=[], help="extra -D definitions")
    ap.add_argument("--src", default=None, help="dev variant source (must sit in csrc/ for its includes)")
    a = ap.parse_args()
    build(force=a.force, out=a.out, extra=[f"-D{d}" for d in a.defs], src=a.src)
