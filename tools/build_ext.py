#!/usr/bin/env python3
"""In-tree build of the native extensions (no torch JIT cache, no hipify step).

* ``routest_amd/_C*.so``  — gfx950 HIP kernels (csrc/*.hip, hipcc --offload-arch=gfx950) + the
  torch binding TU (csrc/bindings.cpp).  Loaded by :mod:`routest_amd.ops`.
* ``routest_amd/_rt*.so`` — CPU-only C++ runtime (csrc/runtime/*.cpp, g++ + pybind11):
  /predict JSON packing + response formatting, ISO parsing, greedy-CVRP and A* CPU fallbacks.
  Works on machines without a GPU.
* ``build/native/rt_selftest_asan`` (``--sanitize``) — the runtime core built host-only with
  ``-fsanitize=address,undefined`` into a fuzz/self-test executable.

Incremental: an object is rebuilt only when its source or any header is newer.
Usage: ``python tools/build_ext.py [--force] [--jobs N] [--only C|rt|sanitize] [--sanitize]``.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "routest_amd")
BUILD = os.path.join(ROOT, "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdir, abi


def _newer(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: List[str]) -> None:
    print("+", " ".join(cmd[:6]), "...", cmd[-1], flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise SystemExit(f"build failed: {' '.join(cmd)}")


NO_SLP = {"eta_mlp_fwd.hip"}
# host code that must round exactly like Python (csrc/runtime/route_core.h): no FMA contraction
NO_CONTRACT = {"native_server.hip", "route_service.hip", "cch.hip"}
# builtin MFMAs write VGPRs: train_bwd_kernel pins its 256 dW2 accumulators to the AGPRs (inline-asm
# MFMAs), and with the default heuristic the builtin MFMAs beside them also took AGPR destinations,
# which made the allocator park accumulator tiles in VGPRs and copy them around every MFMA
MFMA_VGPR = {"eta_mlp_train.hip"}


def build_C(force: bool = False, jobs: int = 8) -> str:
    inc, libdir, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            # the MLP kernels write their packed-f32 VALU explicitly; the SLP vectoriser would
            # otherwise re-pack scalar f32 FMAs beside MFMAs into v_pk_fma_f32, which costs ~5x its
            # issue slot there (MI355X_MICROARCH.md, "price of one filler")
            extra = ["-fno-slp-vectorize"] if os.path.basename(src) in NO_SLP else []
            if os.path.basename(src) in NO_CONTRACT:
                extra.append("-ffp-contract=off")
            if os.path.basename(src) in MFMA_VGPR:
                extra += ["-mllvm", "-amdgpu-mfma-vgpr-form"]
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", *common, *extra, "-munsafe-fp-atomics",
                              "-I", CSRC, "-I", os.path.join(ROCM, "include"), "-c", src, "-o", obj])
    # torch binding translation units: csrc/bindings.cpp (the module) + csrc/*_bindings.cpp
    for bsrc in sorted(glob.glob(os.path.join(CSRC, "*.cpp"))):
        bobj = os.path.join(BUILD, os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if force or _newer(bobj, [bsrc] + headers):
            cmd = [hipcc, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                   "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                   "-I", CSRC, "-I", py_inc]
            for d in inc:
                cmd += ["-I", d]
            cmd += ["-Wno-unused-result", "-Wno-deprecated-declarations", "-c", bsrc, "-o", bobj]
            jobs_list.append(cmd)
    with ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    out = os.path.join(PKG, "_C" + EXT_SUFFIX)
    if force or jobs_list or _newer(out, objs):
        # RCCL: link the copy torch itself loads (torch/lib/librccl.so, no SONAME) so one RCCL
        # instance serves both torch.distributed and our own communicators
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-L", libdir, "-o", out, *objs,
              "-L", libdir, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              "-ltorch_python", "-lamdhip64", "-l:librccl.so", f"-Wl,-rpath,{libdir}"])
    return out


def build_rt(force: bool = False, jobs: int = 8) -> str:
    import pybind11
    py_inc = sysconfig.get_paths()["include"]
    srcs = sorted(p for p in glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))
                  if not p.endswith("_selftest.cpp"))
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    out = os.path.join(PKG, "_rt" + EXT_SUFFIX)
    if not srcs:
        return ""
    if force or _newer(out, srcs + headers):
        _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-pthread",
              "-ffp-contract=off",
              "-I", pybind11.get_include(), "-I", py_inc, "-I", os.path.join(CSRC, "runtime"),
              *srcs, "-o", out])
    return out


def build_sanitize(force: bool = False, kind: str = "asan") -> str:
    """Host-only sanitizer builds of the runtime core fuzz harness (no GPU code involved):
    ``asan`` = AddressSanitizer + UBSan, ``tsan`` = ThreadSanitizer (parallel pack/format paths)."""
    rdir = os.path.join(CSRC, "runtime")
    src = os.path.join(rdir, "rt_selftest.cpp")
    out = os.path.join(BUILD, f"rt_selftest_{kind}")
    os.makedirs(BUILD, exist_ok=True)
    flags = (["-fsanitize=address,undefined", "-fno-sanitize-recover=all"] if kind == "asan"
             else ["-fsanitize=thread"])
    if force or _newer(out, [src] + glob.glob(os.path.join(rdir, "*.h"))):
        _run(["g++", "-std=c++17", "-O1", "-g", *flags, "-fno-omit-frame-pointer", "-pthread", "-I", rdir, src,
              "-o", out, "-ldl"])
    return out


def build_tools(force: bool = False) -> str:
    """Host-only helper executables (build/native/loadgen: closed-loop HTTP load generator)."""
    src = os.path.join(CSRC, "tools", "loadgen.cpp")
    out = os.path.join(BUILD, "loadgen")
    os.makedirs(BUILD, exist_ok=True)
    if force or _newer(out, [src, os.path.join(CSRC, "runtime", "http_client.h")]):
        _run(["g++", "-O2", "-std=c++17", "-pthread", src, "-o", out])
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", choices=["C", "rt", "sanitize", "tools"], default=None)
    ap.add_argument("--sanitize", action="store_true", help="also build the ASan/UBSan runtime harness")
    a = ap.parse_args()
    if a.only == "sanitize" or a.sanitize:
        print("built", build_sanitize(a.force, "asan"))
        print("built", build_sanitize(a.force, "tsan"))
        if a.only == "sanitize":
            return
    if a.only in (None, "tools"):
        print("built", build_tools(a.force))
    if a.only in (None, "rt"):
        print("built", build_rt(a.force, a.jobs))
    if a.only in (None, "C"):
        print("built", build_C(a.force, a.jobs))


if __name__ == "__main__":
    main()
