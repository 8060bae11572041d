"""Loader of the native engine module.

The extension is built in-tree (``python -m mxstream.build``). Importing it never silently falls
back to Python: if the module is missing it is built on the spot (CPU-side cross-compile takes
~10 s); if that fails the import error is raised.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def load():
    """Return the `_mxs_native` module, building it if necessary."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module("mxstream._mxs_native")
        except ImportError:
            if os.environ.get("MXS_NO_AUTOBUILD"):
                raise
            from mxstream import build as _build

            _build.build()
            _mod = importlib.import_module("mxstream._mxs_native")
        return _mod


def loaded_path() -> str:
    return load().__file__
