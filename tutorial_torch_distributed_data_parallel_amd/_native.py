"""Loader for the in-tree native extension (``_C*.so``, built by ``_build.py``).

Policy: GPU tensors always run on the native gfx950 kernels. If the extension is missing or fails
to load, any GPU op raises :class:`NativeUnavailable` -- there is no silent fallback to ATen on a
GPU. CPU tensors (the gloo/CPU plumbing config and the unit tests) use the plain PyTorch
reference implementations in ``ops/``.
"""
from __future__ import annotations

import importlib
import os

_mod = None
_err: Exception | None = None


class NativeUnavailable(RuntimeError):
    pass


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    try:
        import torch  # noqa: F401  (must be loaded first: provides libamdhip64 / librccl)

        _mod = importlib.import_module(f"{__package__}._C")
    except Exception as e:  # pragma: no cover - depends on the build state
        if os.environ.get("TDP_AUTOBUILD", "1") == "1":
            try:
                from . import _build

                _build.build()
                _mod = importlib.import_module(f"{__package__}._C")
                return
            except Exception as e2:  # noqa: BLE001
                _err = e2
                return
        _err = e


def available() -> bool:
    _load()
    return _mod is not None


def native():
    """The extension module; raises if it cannot be loaded."""
    _load()
    if _mod is None:
        raise NativeUnavailable(
            f"native gfx950 extension unavailable ({_err!r}); build it with "
            f"`python -m {__package__}._build`")
    return _mod


def so_file() -> str | None:
    _load()
    return getattr(_mod, "__file__", None) if _mod is not None else None
