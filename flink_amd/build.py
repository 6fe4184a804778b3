"""Builds flink_amd/libgpuwin.so (gfx950) in-tree with hipcc.

    python -m flink_amd.build [--force] [--jobs N]

Sources: flink_amd/csrc/*.hip (kernels) + gw_runtime.cpp (host runtime + C ABI of
include/gpuwin.h).  No torch in the library: it links the HIP runtime and RCCL (gw_exchange.cpp).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgpuwin.so")
OBJDIR = os.path.join(HERE, "_build")
SOURCES = ["gw_pane.hip", "gw_keygroups.hip", "gw_sort.hip", "gw_session.hip", "gw_netbuf.hip", "gw_first.hip", "gw_select.hip", "gw_runtime.cpp",
           "gw_exchange.cpp"]
ROCM_LIB = os.environ.get("ROCM_PATH", "/opt/rocm") + "/lib"
ARCH = os.environ.get("GW_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", f"--offload-arch={ARCH}",
          "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result"]


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(os.path.dirname(HERE), "include", "gpuwin.h"))
    return hs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, force, defines=(), objdir=OBJDIR):
    obj = os.path.join(objdir, src + ".o")
    deps = [os.path.join(CSRC, src)] + _headers()
    if not force and not _stale(obj, deps):
        return obj, None
    cmd = [HIPCC, *CFLAGS, *[f"-D{d}" for d in defines], "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(force: bool = False, jobs: int = 4, verbose: bool = False, defines=(), out: str = OUT) -> str:
    """defines/out: experiment builds (-D knobs into another .so, loaded through GW_LIB_PATH)."""
    objdir = OBJDIR if not defines else os.path.join(OBJDIR, "exp_" + os.path.basename(out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force or bool(defines), defines, objdir), SOURCES))
    errors = [e for _, e in results if e]
    if errors:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errors))
    objs = [o for o, _ in results]
    if force or defines or _stale(out, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs, f"-L{ROCM_LIB}", "-lrccl",
               f"-Wl,-rpath,{ROCM_LIB}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--define", action="append", default=[], help="experiment build: -D knob (needs --out)")
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    try:
        build(args.force, args.jobs, verbose=True, defines=args.define, out=os.path.abspath(args.out))
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
