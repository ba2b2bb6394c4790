"""Weights-only reader for the original-NeRF ``.npy`` weight files.

``data/lego_example_weights/model_200000.npy`` and ``model_fine_200000.npy`` in
the reference are ``np.save`` of an object array (``descr '|O'``, shape (24,)),
so past the ``.npy`` header the file is a pickle stream.  ``np.load`` refuses it
with ``allow_pickle=False``.  This module reads it WITHOUT unpickling: the stream
is walked opcode by opcode with ``pickletools.genops`` (a disassembler, which
executes nothing), and a small stack machine of our own interprets only the
opcodes an ndarray pickle uses.

* A ``GLOBAL`` / ``STACK_GLOBAL`` is never resolved or imported.  Its
  ``module.name`` string is checked against ``ALLOWED_GLOBALS`` (the four names
  an ndarray pickle references: ``numpy.core.multiarray._reconstruct`` -- or its
  numpy-2 path ``numpy._core...`` --, ``numpy.ndarray``, ``numpy.dtype``,
  ``_codecs.encode``) and anything else raises
  ``RefusedPickle`` before the stream is interpreted any further.
* ``REDUCE`` / ``BUILD`` are interpreted symbolically for exactly those four
  names: ``_codecs.encode(s, 'latin1')`` becomes ``s.encode('latin1')``,
  ``numpy.dtype(spec, 0, 1)`` becomes a plain numeric dtype (or the object-array
  marker), ``_reconstruct(ndarray, (0,), b'b')`` becomes an empty array
  placeholder whose ``BUILD`` state ``(version, shape, dtype, fortran, raw)`` is
  turned into ``np.frombuffer(raw, dtype).reshape(shape)``.
* Every other opcode raises ``RefusedPickle``.

So the reader is a data parser: nothing in the file can name code that runs.
"""
from __future__ import annotations

import pickletools
from typing import Any, List

import numpy as np

ALLOWED_GLOBALS = frozenset({
    "numpy.core.multiarray._reconstruct",
    "numpy._core.multiarray._reconstruct",     # the same function as numpy >= 2 names it
    "numpy.ndarray",
    "numpy.dtype",
    "_codecs.encode",
})

# plain numeric dtypes the weights may use; 'O8' is the outer object array
_NUMERIC = {"f2", "f4", "f8", "i1", "i2", "i4", "i8", "u1", "u2", "u4", "u8", "b1"}


class RefusedPickle(ValueError):
    """The stream names a global or an opcode outside the ndarray subset."""


class _Global:
    def __init__(self, qual: str):
        self.qual = qual


class _Dtype:
    def __init__(self, spec: str):
        self.spec = spec
        self.order = "|"

    def resolve(self):
        if self.spec == "O8":
            return "object"
        dt = np.dtype(self.spec)
        return dt.newbyteorder(self.order) if self.order in "<>" else dt


class _ArrayStub:
    def __init__(self):
        self.value = None


class _Mark:
    pass


_MARK = _Mark()


def _reduce(func: Any, args: tuple):
    if not isinstance(func, _Global):
        raise RefusedPickle("REDUCE on a non-global callable")
    q = func.qual
    if q == "_codecs.encode":
        if len(args) != 2 or not isinstance(args[0], str) or args[1] != "latin1":
            raise RefusedPickle(f"_codecs.encode{args!r:.60}")
        return args[0].encode("latin1")
    if q == "numpy.dtype":
        if len(args) != 3 or not isinstance(args[0], str) or (args[0] not in _NUMERIC and args[0] != "O8"):
            raise RefusedPickle(f"numpy.dtype{args!r:.60}")
        return _Dtype(args[0])
    if q in ("numpy.core.multiarray._reconstruct", "numpy._core.multiarray._reconstruct"):
        if (len(args) != 3 or not isinstance(args[0], _Global) or args[0].qual != "numpy.ndarray"
                or args[1] != (0,)):
            raise RefusedPickle(f"_reconstruct{args!r:.60}")
        return _ArrayStub()
    raise RefusedPickle(f"REDUCE of {q}")


def _build(obj: Any, state: Any):
    if isinstance(obj, _Dtype):
        if not isinstance(state, tuple) or len(state) < 2 or state[1] not in ("<", ">", "|", "="):
            raise RefusedPickle("dtype state")
        obj.order = state[1]
        return obj
    if isinstance(obj, _ArrayStub):
        if not isinstance(state, tuple) or len(state) != 5:
            raise RefusedPickle("ndarray state")
        _, shape, dt, fortran, raw = state
        if not isinstance(dt, _Dtype) or not isinstance(shape, tuple):
            raise RefusedPickle("ndarray state")
        kind = dt.resolve()
        if kind == "object":
            if not isinstance(raw, list) or len(raw) != int(np.prod(shape)):
                raise RefusedPickle("object-array state")
            obj.value = list(raw)
        else:
            if not isinstance(raw, (bytes, bytearray)):
                raise RefusedPickle("ndarray payload")
            a = np.frombuffer(bytes(raw), dtype=kind)
            obj.value = a.reshape(shape, order="F" if fortran else "C").astype(kind.newbyteorder("="), copy=True)
        return obj
    raise RefusedPickle(f"BUILD on {type(obj).__name__}")


def _value(x):
    return x.value if isinstance(x, _ArrayStub) else x


def parse_pickle(data: bytes) -> Any:
    """Interpret an ndarray pickle stream (see the module docstring)."""
    try:
        ops = list(pickletools.genops(data))
    except Exception as e:                     # malformed stream
        raise RefusedPickle(f"not a well-formed pickle stream: {e}") from None
    # refuse on names before interpreting anything
    for op, arg, _ in ops:
        if op.name == "GLOBAL":
            qual = arg.replace(" ", ".")
            if qual not in ALLOWED_GLOBALS:
                raise RefusedPickle(f"global {qual!r} is not in the ndarray allowlist")
    stack: List[Any] = []
    memo = {}
    for op, arg, _ in ops:
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "GLOBAL":
            stack.append(_Global(arg.replace(" ", ".")))
        elif n == "STACK_GLOBAL":
            name, mod = stack.pop(), stack.pop()
            qual = f"{mod}.{name}"
            if qual not in ALLOWED_GLOBALS:
                raise RefusedPickle(f"global {qual!r} is not in the ndarray allowlist")
            stack.append(_Global(qual))
        elif n in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "MARK":
            stack.append(_MARK)
        elif n == "TUPLE":
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            items = tuple(stack[k + 1:])
            del stack[k:]
            stack.append(items)
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(_value(v))
        elif n == "APPENDS":
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[k + 1:]
            del stack[k:]
            if not isinstance(stack[-1], list):
                raise RefusedPickle("APPENDS to a non-list")
            stack[-1].extend(_value(v) for v in items)
        elif n in ("BININT", "BININT1", "BININT2"):
            stack.append(int(arg))
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n in ("BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8"):
            stack.append(str(arg))
        elif n in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            if not isinstance(args, tuple):
                raise RefusedPickle("REDUCE without an argument tuple")
            stack.append(_reduce(func, args))
        elif n == "BUILD":
            state = stack.pop()
            stack[-1] = _build(stack[-1], state)
        elif n == "STOP":
            if len(stack) != 1:
                raise RefusedPickle("malformed stream")
            return _value(stack[0])
        else:
            raise RefusedPickle(f"opcode {n} is outside the ndarray subset")
    raise RefusedPickle("stream has no STOP")


def read_object_npy(path: str) -> List[np.ndarray]:
    """The arrays of an ``np.save``'d object array, read without unpickling."""
    with open(path, "rb") as f:
        version = np.lib.format.read_magic(f)
        if version == (1, 0):
            shape, _, dtype = np.lib.format.read_array_header_1_0(f)
        else:
            shape, _, dtype = np.lib.format.read_array_header_2_0(f)
        if dtype != np.dtype("O"):
            raise RefusedPickle(f"{path}: dtype {dtype} is not an object array")
        data = f.read()
    out = parse_pickle(data)
    if not isinstance(out, list) or len(out) != int(np.prod(shape)):
        raise RefusedPickle(f"{path}: expected {shape} arrays")
    for a in out:
        if not isinstance(a, np.ndarray):
            raise RefusedPickle(f"{path}: element is not an ndarray")
    return out
