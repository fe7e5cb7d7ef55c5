"""Build the native modules in-tree.

* ``_sphx_cpu``  — OpenMP reference path, compiled with g++ (same libgomp as PyTorch).
* ``_sphx_hip``  — gfx950 kernels + host launchers, compiled with hipcc ``--offload-arch=gfx950``.
* ``_sphx_io``   — H5Part-compatible HDF5 reader/writer linked against the image's serial libhdf5.

Outputs land in ``sphexa_amd/_native/`` so they travel with the repository snapshot to the GPU box.
Builds are incremental (object files are rebuilt only when a source or header is newer).
"""

from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_native")
OBJ = os.path.join(OUT, "obj")
EXT = sysconfig.get_config_var("EXT_SUFFIX")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HDF5_ROOT = os.environ.get("SPHX_HDF5_ROOT", "/opt/conda")
ARCH = os.environ.get("SPHX_OFFLOAD_ARCH", "gfx950")


def _py_includes():
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _headers():
    return glob.glob(os.path.join(CSRC, "include", "sphx", "*.hpp")) + glob.glob(os.path.join(CSRC, "*", "*.hpp"))


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _flags_changed(obj_dir, tag, flags):
    """True (and records the new set) if the compile flags of ``tag`` differ from the last build's"""
    stamp = os.path.join(obj_dir, f".{tag}.flags")
    cur = " ".join(flags)
    old = open(stamp).read() if os.path.exists(stamp) else None
    if old != cur:
        with open(stamp, "w") as f:
            f.write(cur)
        return True
    return False


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _compile_all(jobs, verbose):
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        futs = {ex.submit(_run, cmd): out for cmd, out in jobs}
        for f in cf.as_completed(futs):
            f.result()
            if verbose:
                print(f"  built {os.path.basename(futs[f])}", flush=True)


def _cpu_march():
    try:
        with open("/proc/cpuinfo") as f:
            flags = f.read()
        if " avx2 " in flags and " fma " in flags:
            return ["-march=x86-64-v3"]
    except OSError:
        pass
    return []


SANITIZE_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]


def build_cpu(verbose=False, sanitize=False):
    """``sanitize``: AddressSanitizer + UBSan build of the OpenMP module into _native/sanitize/ (loaded when
    SPHX_CPU_VARIANT=sanitize; the process needs libasan preloaded, see tests/test_sanitize.py)"""
    out_dir = os.path.join(OUT, "sanitize") if sanitize else OUT
    obj_dir = os.path.join(out_dir, "obj") if sanitize else OBJ
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "cpu", "*.cpp")))
    target = os.path.join(out_dir, "_sphx_cpu" + EXT)
    opt = ["-O1", "-g"] + SANITIZE_FLAGS if sanitize else ["-O3"] + _cpu_march()
    flags = opt + ["-std=c++17", "-fPIC", "-fopenmp", f"-I{os.path.join(CSRC, 'include')}",
                   f"-I{os.path.join(CSRC, 'cpu')}"] + _py_includes()
    hdrs = _headers()
    force = _flags_changed(obj_dir, "cpu", flags)
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(obj_dir, "cpu_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs.append((["g++", *flags, "-c", s, "-o", o], o))
    _compile_all(jobs, verbose)
    if jobs or _newer(target, objs):
        _run(["g++", "-shared", "-fopenmp", *(SANITIZE_FLAGS if sanitize else []), *objs, "-o", target])
    return target


def build_hip(verbose=False, variant=None, defines=()):
    """``variant``/``defines``: tuning build into _native/variants/<variant>/ with extra -D flags (loaded when
    SPHX_HIP_VARIANT=<variant> is set)"""
    out_dir = os.path.join(OUT, "variants", variant) if variant else OUT
    obj_dir = os.path.join(out_dir, "obj") if variant else OBJ
    os.makedirs(obj_dir, exist_ok=True)
    hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")) + glob.glob(os.path.join(CSRC, "hip", "*.cpp")))
    target = os.path.join(out_dir, "_sphx_hip" + EXT)
    # fp32 division/sqrt as the hardware rcp/sqrt (<= 1 ulp) instead of the IEEE correctly-rounded expansions
    # (~10 VALU each): the SPH pair loops are VALU-bound on MI355X (profiles/), the results stay fp32-accurate.
    # No SLP vectorization: its v_pk_*_f32 pairs cost operand-packing moves and registers in the pair loops
    # (A/B: Sedov -n 400 192 -> 183 ms/step, momentum/energy 45 -> 40 ms; Evrard -n 200 41.6 -> 40.2 ms)
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize",
             f"-I{os.path.join(CSRC, 'include')}", f"-I{os.path.join(CSRC, 'hip')}"] + list(defines) + _py_includes()
    hdrs = _headers() + glob.glob(os.path.join(CSRC, "hip", "*.h"))
    force = _flags_changed(obj_dir, "hip", flags)
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(obj_dir, "hip_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            jobs.append(([hipcc, *flags, *lang, "-c", s, "-o", o], o))
    _compile_all(jobs, verbose)
    if jobs or _newer(target, objs):
        # link to a temporary name and rename: a concurrent reader (a repository snapshot, a running test) sees the
        # old or the new module, never a partial one
        tmp = target + ".tmp"
        _run([hipcc, "-shared", f"--offload-arch={ARCH}", *objs, "-o", tmp,
              f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"])
        os.replace(tmp, target)
    return target


def build_io(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "io", "*.cpp")))
    if not srcs or not os.path.exists(os.path.join(HDF5_ROOT, "include", "hdf5.h")):
        return None
    target = os.path.join(OUT, "_sphx_io" + EXT)
    flags = ["-O2", "-std=c++17", "-fPIC", f"-I{HDF5_ROOT}/include", f"-I{os.path.join(CSRC, 'include')}"] + \
        _py_includes()
    jobs, objs = [], []
    for s in srcs:
        o = os.path.join(OBJ, "io_" + os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(o, [s] + _headers()):
            jobs.append((["g++", *flags, "-c", s, "-o", o], o))
    _compile_all(jobs, verbose)
    if jobs or _newer(target, objs):
        # link libhdf5 by full path with an rpath so that the conda lib directory is not put in front of the
        # system libraries for everything else in the process
        _run(["g++", "-shared", *objs, "-o", target, os.path.join(HDF5_ROOT, "lib", "libhdf5.so.103"),
              f"-Wl,-rpath,{HDF5_ROOT}/lib"])
    return target


def build_golden(verbose=False):
    """fp64 instantiation of the SPH j-loops (golden-value tests, csrc/golden/golden.cpp)"""
    os.makedirs(OBJ, exist_ok=True)
    src = os.path.join(CSRC, "golden", "golden.cpp")
    target = os.path.join(OUT, "_sphx_golden" + EXT)
    flags = ["-O2", "-std=c++17", "-fPIC", "-DSPHX_HYDRO_TYPE=double", f"-I{os.path.join(CSRC, 'include')}"] + \
        _py_includes()
    if _newer(target, [src] + _headers()) or _flags_changed(OBJ, "golden", flags):
        _run(["g++", *flags, "-shared", src, "-o", target])
        if verbose:
            print("  built _sphx_golden", flush=True)
    return target


def build_all(verbose=False, hip=True):
    out = [build_cpu(verbose), build_io(verbose), build_golden(verbose)]
    if hip:
        out.append(build_hip(verbose))
    return [o for o in out if o]


def build_dcheck(verbose=False):
    """device-check build of the HIP module (csrc/hip/common.h SPHX_DCHECK) into _native/variants/dcheck/, loaded
    when SPHX_DEVICE_CHECKS=1: failed range checks are flagged and reported after the step instead of faulting"""
    return build_hip(verbose=verbose, variant="dcheck", defines=["-DSPHX_DEVICE_CHECKS"])


if __name__ == "__main__":
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        tag = sys.argv[i + 1]
        defs = [a for a in sys.argv[i + 2:] if a.startswith(("-D", "-f", "-m"))]
        print("ok", build_hip(verbose=True, variant=tag, defines=defs))
        sys.exit(0)
    if "--sanitize" in sys.argv:
        print("ok", build_cpu(verbose=True, sanitize=True))
        sys.exit(0)
    if "--dcheck" in sys.argv:
        print("ok", build_dcheck(verbose=True))
        sys.exit(0)
    skip_hip = "--no-hip" in sys.argv
    for t in build_all(verbose=True, hip=not skip_hip):
        print("ok", t)
