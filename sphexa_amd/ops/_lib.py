"""Loader for the in-tree native modules.

The HIP module is mandatory whenever a GPU is present: an op on a CUDA(HIP) tensor never silently falls back to
PyTorch or the CPU path — it raises if ``_sphx_hip`` cannot be loaded.
"""

from __future__ import annotations

import importlib.util
import os
import sys
import sysconfig

_NATIVE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")
_EXT = sysconfig.get_config_var("EXT_SUFFIX")
_cache: dict = {}


def _load(name: str):
    if name in _cache:
        return _cache[name]
    path = os.path.join(_NATIVE_DIR, name + _EXT)
    variant = os.environ.get("SPHX_HIP_VARIANT") if name == "_sphx_hip" else None
    if name == "_sphx_hip" and os.environ.get("SPHX_DEVICE_CHECKS") == "1":
        variant = "dcheck"  # device-check build (build_native --dcheck)
    if name == "_sphx_cpu" and os.environ.get("SPHX_CPU_VARIANT") == "sanitize":
        # ASan/UBSan build of the OpenMP module (build_native --sanitize)
        path = os.path.join(_NATIVE_DIR, "sanitize", name + _EXT)
        if not os.path.exists(path):
            raise ImportError(f"sanitizer build not found: {path} (python -m sphexa_amd.build_native --sanitize)")
    elif variant:
        # tuning builds: sphexa_amd/_native/variants/<tag>/_sphx_hip*.so (build_native --variant tag -DNAME=V ...)
        path = os.path.join(_NATIVE_DIR, "variants", variant, name + _EXT)
        if not os.path.exists(path):
            raise ImportError(f"HIP variant {variant} not built: {path}")
    if not os.path.exists(path):
        # build on first use (CPU container or fresh checkout)
        from .. import build_native

        if name == "_sphx_cpu":
            build_native.build_cpu()
        elif name == "_sphx_hip":
            build_native.build_hip()
        elif name == "_sphx_io":
            build_native.build_io()
        elif name == "_sphx_golden":
            build_native.build_golden()
    if not os.path.exists(path):
        raise ImportError(f"native module {name} not found at {path}")
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules[name] = mod
    _cache[name] = mod
    return mod


def cpu():
    return _load("_sphx_cpu")


def hip():
    return _load("_sphx_hip")


def io():
    return _load("_sphx_io")


def golden():
    return _load("_sphx_golden")


def native_paths():
    """the .so files this process has loaded (for diagnostics / smoke tests)"""
    return {k: getattr(v, "__file__", None) for k, v in _cache.items()}


class DeviceCheckError(RuntimeError):
    """a device-side check of the SPHX_DEVICE_CHECKS build failed (see csrc/hip/common.h for the bits)"""


DEVICE_CHECK_BITS = {0: "neighbor index out of range", 1: "list blocks of a group above the maximum",
                     2: "gather permutation index out of range", 3: "gravity interaction list longer than its slab",
                     4: "halo pack index out of range", 5: "search band re-test source index out of range"}


def raise_on_device_check(where: str = ""):
    """with SPHX_DEVICE_CHECKS=1 (device-check HIP build loaded): raise if any device check failed since the last
    call. A no-op otherwise (no device synchronization)."""
    if os.environ.get("SPHX_DEVICE_CHECKS") != "1" or "_sphx_hip" not in _cache:
        return
    flags = int(_cache["_sphx_hip"].device_check_flags())
    if flags:
        names = [v for b, v in DEVICE_CHECK_BITS.items() if flags >> b & 1]
        raise DeviceCheckError(f"device checks failed{(' in ' + where) if where else ''}: {', '.join(names)} "
                               f"(flags {flags:#x})")


try:  # the raw current-stream query torch's own generated launch code uses (no Stream object, no device checks)
    from torch._C import _cuda_getCurrentRawStream as _raw_stream, _cuda_getDevice as _cur_dev
except ImportError:  # pragma: no cover
    _raw_stream = _cur_dev = None


def stream() -> int:
    """the current HIP stream of the current device as an integer handle for the native launchers: what
    ``torch.cuda.current_stream().cuda_stream`` returns (a ``with torch.cuda.stream(...)`` block included), without
    building a Stream object (~0.3 instead of ~4 us per launch; ~40 launches per step)"""
    if _raw_stream is not None:
        return _raw_stream(_cur_dev())
    import torch

    return torch.cuda.current_stream().cuda_stream
