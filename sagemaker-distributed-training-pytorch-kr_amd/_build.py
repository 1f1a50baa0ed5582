"""In-tree native build for smdt_amd (no pip install, no JIT cache under ~/.cache).

Produces, next to this file:
  * ``_C.so``       - the gfx950 HIP kernel library + PyTorch bindings (hipcc, ``--offload-arch=gfx950``)
  * ``_runtime.so`` - host-side C++ runtime (GPT index builders, process supervisor helpers),
                      pybind11 only, no torch and no HIP.

Kernel translation units are compiled WITHOUT PyTorch headers (seconds each) and only
``bindings.cpp`` pulls ATen in. Objects are rebuilt when their source or any header changed;
compilation runs in a thread pool. We drive hipcc directly instead of
``torch.utils.cpp_extension`` so no hipify pass ever touches the sources.

Usage: ``python -m smdt_amd._build`` (or ``python setup.py build_ext``; ``__graft_entry__.build()``).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
ARCH = os.environ.get("SMDT_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
CXX = shutil.which("g++") or "c++"


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    incs = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames else ce.include_paths(True)
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libdir, abi


def _py_includes():
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _newer(src_files, out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


# Per-file device-compiler flags (measured choices). flash_attn: the SLP vectorizer packs the
# softmax f32 math into v_pk_*_f32, which pins register pairs and measured 4 % slower in the
# backward (profiles/r1_attn_dropout/ab_attention.log).
KERNEL_FLAGS = {"flash_attn.hip": ["-fno-slp-vectorize"]}


def kernel_sources():
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def build_kernels(verbose=False, jobs=None):
    """Compile every HIP kernel TU + bindings and link ``_C.so``."""
    os.makedirs(BUILD, exist_ok=True)
    incs, libdir, abi = _torch_paths()
    hdrs = headers()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", os.path.join(CSRC, "kernels"),
              "-Wno-unused-result", "-Wno-pass-failed"]
    # SMDT_KERNEL_FLAGS="file.hip:-flag,-flag;other.hip:-flag" adds per-file flags (A/B builds);
    # the object name carries a hash of them so a flag change forces a rebuild.
    extra = dict(KERNEL_FLAGS)
    for item in filter(None, os.environ.get("SMDT_KERNEL_FLAGS", "").split(";")):
        f, _, fl = item.partition(":")
        extra[f.strip()] = [x for x in fl.split(",") if x]
    jobs_list = []
    objs = []
    for src in kernel_sources():
        base = os.path.basename(src)
        fl = extra.get(base, [])
        tag = ("." + hashlib.sha1(" ".join(fl).encode()).hexdigest()[:8]) if fl else ""
        obj = os.path.join(BUILD, base + tag + ".o")
        objs.append(obj)
        if _newer([src] + hdrs, obj):
            jobs_list.append([HIPCC] + common + fl + ["-c", src, "-o", obj])
    # Host TUs that include ATen (bindings, hipBLASLt plans): compiled by hipcc so HIP headers
    # resolve; no device code in them.
    binc = []
    for d in incs + _py_includes():
        binc += ["-I", d]
    for bsrc in sorted(glob.glob(os.path.join(CSRC, "*.cpp"))):
        bobj = os.path.join(BUILD, os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if _newer([bsrc] + hdrs, bobj):
            jobs_list.append([HIPCC, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
                              "-DTORCH_API_INCLUDE_EXTENSION_H", "-I", CSRC, "-Wno-deprecated-declarations",
                              "-Wno-unused-result"] + binc + ["-c", bsrc, "-o", bobj])
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs_list))
    out = os.path.join(HERE, "_C.so")
    if jobs_list or not os.path.exists(out):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs + [
            "-L", libdir, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-l:libhipblaslt.so",
            f"-Wl,-rpath,{libdir}"]
        _run(link, verbose)
    return out


def build_runtime(verbose=False):
    """Compile the host C++ runtime (pybind11, no torch) into ``_runtime.so``."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return None
    out = os.path.join(HERE, "_runtime" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    alias = os.path.join(HERE, "_runtime.so")
    if _newer(srcs + headers(), out):
        inc = []
        for d in _py_includes():
            inc += ["-I", d]
        _run([CXX, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I", CSRC] + inc + srcs + ["-o", out, "-lpthread"], verbose)
    if out != alias:
        try:
            if os.path.islink(alias) or os.path.exists(alias):
                os.remove(alias)
        except OSError:
            pass
    return out


SANITIZE_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                  "-fno-sanitize-recover=undefined"]


def build_runtime_sanitized(out_dir, verbose=False):
    """Build the host runtime with AddressSanitizer + UBSan into ``out_dir/_runtime.so``
    (SURVEY §5.2 "address-sanitizer build target"). Host code only: GPU ASan is not used.

    The module must be imported by a Python started with ``LD_PRELOAD`` of
    ``sanitizer_preload()`` (``scripts/sanitize_runtime.py`` does this)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "_runtime" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    if _newer(srcs + headers(), out):
        inc = []
        for d in _py_includes():
            inc += ["-I", d]
        _run([CXX, "-std=c++17", "-fPIC", "-shared", "-Wall"] + SANITIZE_FLAGS + ["-I", CSRC] + inc + srcs
             + ["-o", out, "-lpthread"], verbose)
    return out


def sanitizer_preload():
    """Runtime libraries that must be preloaded into the interpreter for a sanitized module."""
    libs = []
    for name in ("libasan.so", "libubsan.so"):
        p = subprocess.run([CXX, f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
        if p and os.path.isabs(p) and os.path.exists(p):
            libs.append(os.path.realpath(p))
    return libs


def build_all(verbose=False):
    rt = build_runtime(verbose)
    k = build_kernels(verbose)
    return k, rt


if __name__ == "__main__":
    v = "-v" in sys.argv
    print(build_all(verbose=v))
