"""Code-free, typed encoding of host operator state for checkpoints (replaces pickle).

A host operator's snapshot is a tree of Python values: keyed-state tables by key group
(``{key_group: {state name: {(key, namespace): value}}}``, api/state.py), timers, watermarks,
and the values themselves -- Flink ``TupleN`` records, ``TimeWindow`` namespaces, accumulators
(numbers, lists, tuples), numpy columns of the native operators. Flink writes these with typed
serializers (chapter3/README.md:454-456 promises checkpoints/savepoints); this
module does the same with a closed set of tags, so restoring a checkpoint directory never runs
code from it:

  JSON (``.state.json``): None, bool, str, finite floats, ints in the double-exact range as
  themselves; tagged objects for everything else -- ``{"$i": "<decimal>"}`` big ints,
  ``{"$f": "nan"|"inf"|"-inf"}``, ``{"$b": base64}`` bytes, ``{"$t": [...]}`` tuples,
  ``{"$T": [...]}`` Flink tuples, ``{"$d": [[k, v], ...]}`` dicts with non-string keys,
  ``{"$s": [...]}`` sets, ``{"$W": [start, end]}`` TimeWindow, ``{"$G": 0}`` GlobalWindow,
  ``{"$jd": x}`` / ``{"$jl": x}`` Java Double / Long, ``{"$n": [dtype, value]}`` numpy scalars,
  ``{"$a": "<name>"}`` numpy arrays, ``{"$x": [tag, fields]}`` registered user types.
  numpy arrays (``.state.npz``): numeric / bool / fixed-width string dtypes only, read with
  ``allow_pickle=False``.

Anything else raises TypeError at checkpoint time (name the type and register it with
``register_state_type``), never a silent pickle.
"""
from __future__ import annotations

import base64
import io
import json
import math
from pathlib import Path
from typing import Any, Callable

import numpy as np

_MAX_EXACT = 1 << 53
_USER: dict[str, tuple[type, Callable, Callable]] = {}
_USER_BY_TYPE: dict[type, str] = {}


def register_state_type(cls: type, tag: str, to_fields: Callable[[Any], Any],
                        from_fields: Callable[[Any], Any]) -> None:
    """A user type inside operator state (e.g. an accumulator class): ``to_fields(obj)`` returns
    encodable values, ``from_fields(fields)`` rebuilds the object. The tag names it in files."""
    _USER[tag] = (cls, to_fields, from_fields)
    _USER_BY_TYPE[cls] = tag


class _Enc:
    def __init__(self):
        self.arrays: dict[str, np.ndarray] = {}

    def array(self, a: np.ndarray) -> dict:
        if a.dtype.hasobject:
            raise TypeError("checkpoint state: numpy object arrays are not serialisable")
        name = f"a{len(self.arrays)}"
        self.arrays[name] = np.ascontiguousarray(a)
        return {"$a": name}

    def enc(self, x):  # noqa: C901 -- one branch per tag
        from ..api.tuples import Tuple
        from ..api.windowing import GlobalWindow, TimeWindow
        from ..utils.javafmt import JDouble, JLong

        if x is None or isinstance(x, (bool, str)):
            return x
        t = type(x)
        if t in _USER_BY_TYPE:
            tag = _USER_BY_TYPE[t]
            return {"$x": [tag, self.enc(_USER[tag][1](x))]}
        if isinstance(x, JDouble):
            return {"$jd": self.enc(float(x))}
        if isinstance(x, JLong):
            return {"$jl": self.enc(int(x))}
        if isinstance(x, (int, np.integer)) and not isinstance(x, np.generic):
            return x if -_MAX_EXACT <= x <= _MAX_EXACT else {"$i": str(int(x))}
        if isinstance(x, float) and not isinstance(x, np.generic):
            if math.isfinite(x):
                return x
            return {"$f": "nan" if math.isnan(x) else ("inf" if x > 0 else "-inf")}
        if isinstance(x, np.generic):
            if isinstance(x, np.bool_):
                v = bool(x)
            elif isinstance(x, np.integer):
                v = str(int(x))
            elif isinstance(x, np.floating):
                v = repr(float(x))
            else:
                raise TypeError(f"checkpoint state: numpy scalar {x.dtype} is not serialisable")
            return {"$n": [x.dtype.str, v]}
        if isinstance(x, np.ndarray):
            return self.array(x)
        if isinstance(x, (bytes, bytearray, memoryview)):
            return {"$b": base64.b64encode(bytes(x)).decode()}
        if isinstance(x, Tuple):
            return {"$T": [self.enc(v) for v in x]}
        if isinstance(x, TimeWindow):
            return {"$W": [self.enc(x.start), self.enc(x.end)]}
        if isinstance(x, GlobalWindow):
            return {"$G": 0}
        if t is tuple:
            return {"$t": [self.enc(v) for v in x]}
        if t is list:
            return [self.enc(v) for v in x]
        if isinstance(x, (set, frozenset)):
            return {"$s": [self.enc(v) for v in x]}
        if isinstance(x, dict):
            if all(isinstance(k, str) and not k.startswith("$") for k in x):
                return {k: self.enc(v) for k, v in x.items()}
            return {"$d": [[self.enc(k), self.enc(v)] for k, v in x.items()]}
        raise TypeError(f"checkpoint state: a value of type {t.__module__}.{t.__qualname__} has "
                        "no serializer (mxstream.runtime.statecodec.register_state_type)")


def _dec(x, arrays):  # noqa: C901
    if isinstance(x, list):
        return [_dec(v, arrays) for v in x]
    if not isinstance(x, dict):
        return x
    if len(x) == 1:
        (k, v), = x.items()
        if k.startswith("$"):
            from ..api.tuples import Tuple
            from ..api.windowing import GLOBAL_WINDOW, TimeWindow
            from ..utils.javafmt import JDouble, JLong

            if k == "$i":
                return int(v)
            if k == "$f":
                return float(v)
            if k == "$b":
                return base64.b64decode(v)
            if k == "$t":
                return tuple(_dec(e, arrays) for e in v)
            if k == "$T":
                return Tuple(tuple(_dec(e, arrays) for e in v))
            if k == "$d":
                return {_hashable(_dec(a, arrays)): _dec(b, arrays) for a, b in v}
            if k == "$s":
                return {_hashable(_dec(e, arrays)) for e in v}
            if k == "$W":
                return TimeWindow(_dec(v[0], arrays), _dec(v[1], arrays))
            if k == "$G":
                return GLOBAL_WINDOW
            if k == "$jd":
                return JDouble(_dec(v, arrays))
            if k == "$jl":
                return JLong(_dec(v, arrays))
            if k == "$n":
                dt = np.dtype(v[0])
                if dt.kind == "b":
                    return np.bool_(v[1])
                return dt.type(int(v[1])) if dt.kind in "iu" else dt.type(float(v[1]))
            if k == "$a":
                return arrays[v]
            if k == "$x":
                tag, fields = v
                if tag not in _USER:
                    raise TypeError(f"checkpoint state: unknown registered type {tag!r}")
                return _USER[tag][2](_dec(fields, arrays))
            raise ValueError(f"checkpoint state: unknown tag {k!r}")
    return {k: _dec(v, arrays) for k, v in x.items()}


def _hashable(x):
    return tuple(_hashable(e) for e in x) if type(x) is list else x


def encode(obj) -> tuple[str, dict[str, np.ndarray]]:
    """(JSON text, numpy arrays) of a state tree."""
    e = _Enc()
    tree = e.enc(obj)
    return json.dumps(tree, allow_nan=False, separators=(",", ":")), e.arrays


def decode(text: str, arrays: dict[str, np.ndarray] | None = None):
    return _dec(json.loads(text), arrays or {})


def write_state(path: Path, obj) -> None:
    """``path`` (``….state.json``) plus ``….state.npz`` when the state holds arrays; each file
    written to ``.inprogress`` and renamed."""
    import os

    text, arrays = encode(obj)
    npz = path.with_suffix(".npz")
    if arrays:
        buf = io.BytesIO()
        np.savez(buf, **arrays)
        tmp = npz.with_name(npz.name + ".inprogress")
        tmp.write_bytes(buf.getvalue())
        os.replace(tmp, npz)
    tmp = path.with_name(path.name + ".inprogress")
    tmp.write_text(text)
    os.replace(tmp, path)


def read_state(path: Path):
    npz = path.with_suffix(".npz")
    arrays = {}
    if npz.exists():
        with np.load(npz, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
    return decode(path.read_text(), arrays)
