"""Polynomial reference motion table (imitation reward input).

Mirrors ``playground/common/poly_reference_motion.py`` (``PolyReferenceMotion``):

* ``process`` (:74-146) builds a ``[n_dx, n_dy, n_dtheta, 40, 16]`` coefficient grid from
  ``data/polynomial_coefficients.pkl`` with the grid axes sorted (:124-129),
* ``vel_to_index`` (:148-158) clips the command to the grid range and takes the nearest
  grid index per axis (``argmin |grid - v|``, first index on ties),
* ``get_reference_motion`` (:163-168) evaluates the 40 degree-15 polynomials at
  ``t = (i % nb_steps_in_period) / nb_steps_in_period``.

This module evaluates the polynomials once per phase (fp64) into a phase table; the step
kernel (``csrc/duck_env_kernels.h``) looks the table up by grid cell and phase. The reference stores the table as a pickle. Pickles that ship with the
reference are never unpickled here: :func:`read_poly_pkl` walks the opcode stream with
``pickletools.genops`` and interprets only inert data opcodes (dict/list/str/float/bytes
and the two numpy scalar reconstructors, whose raw bytes are decoded with ``struct``),
so nothing from the file is ever imported or executed.
"""

from __future__ import annotations

import pickletools
import struct
from typing import Any, Dict

import numpy as np

_ALLOWED_GLOBALS = {("numpy.core.multiarray", "scalar"), ("numpy", "dtype"),
                    ("numpy._core.multiarray", "scalar")}


class _Global:
    def __init__(self, mod, name):
        self.key = (mod, name)


class _DType:
    def __init__(self, code):
        self.code = code


_MARK = object()


def read_poly_pkl(path: str) -> Dict[str, Any]:
    """Decode ``polynomial_coefficients.pkl`` without unpickling (data opcodes only)."""
    with open(path, "rb") as f:
        data = f.read()
    stack: list = []
    memo: Dict[int, Any] = {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n == "MARK":
            stack.append(_MARK)
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE", "BINUNICODE8"):
            stack.append(str(arg))
        elif n in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif n in ("BININT1", "BININT2", "BININT", "INT", "LONG1"):
            stack.append(int(arg))
        elif n in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "TUPLE1":
            stack[-1:] = [tuple(stack[-1:])]
        elif n == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif n == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            if (mod, name) not in _ALLOWED_GLOBALS:
                raise ValueError(f"refusing global {mod}.{name}")
            stack.append(_Global(mod, name))
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, _Global):
                raise ValueError("REDUCE on non-global")
            if fn.key == ("numpy", "dtype"):
                stack.append(_DType(args[0]))
            else:  # numpy scalar: (dtype, raw bytes)
                dt, raw = args
                if dt.code != "f8" or len(raw) != 8:
                    raise ValueError(f"unsupported scalar {dt.code}")
                stack.append(struct.unpack("<d", raw)[0])
        elif n == "BUILD":
            stack.pop()  # dtype state tuple: byte order etc. (little-endian f8 checked above)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "APPEND":
            item = stack.pop()
            stack[-1].append(item)
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for k, v in zip(items[::2], items[1::2]):
                d[k] = v
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "STOP":
            break
        else:
            raise ValueError(f"unsupported pickle opcode {n}")
    (out,) = stack
    return out


def bake_table(data: Dict[str, Any]) -> Dict[str, np.ndarray]:
    """Grid the per-command polynomial sets as ``PolyReferenceMotion.process`` does.

    Coefficients are kept in ascending-power order (as stored in the pkl); the reference
    flips them for ``jp.polyval`` (``poly_reference_motion.py:122``), which evaluates the
    same polynomial.
    """
    first = next(iter(data.values()))
    period = float(first["period"])
    fps = float(first["fps"])
    keys = list(data.keys())
    dxs = sorted({float(k.split("_")[0]) for k in keys})
    dys = sorted({float(k.split("_")[1]) for k in keys})
    dths = sorted({float(k.split("_")[2]) for k in keys})
    ndim = len(first["coefficients"])
    ncoef = len(next(iter(first["coefficients"].values())))
    table = np.zeros((len(dxs), len(dys), len(dths), ndim, ncoef), dtype=np.float64)
    filled = np.zeros(table.shape[:3], dtype=bool)
    for k, v in data.items():
        dx, dy, dth = (float(s) for s in k.split("_"))
        ix, iy, it = dxs.index(dx), dys.index(dy), dths.index(dth)
        for d, (_, c) in enumerate(v["coefficients"].items()):
            table[ix, iy, it, d] = np.asarray(c, dtype=np.float64)
        filled[ix, iy, it] = True
    if not filled.all():
        raise ValueError("incomplete reference-motion grid")
    # ranges as the reference computes them: start at [0, 0] and widen (:52-57)
    rng = lambda g: np.array([min(0.0, min(g)), max(0.0, max(g))])
    return dict(coeffs=table, dxs=np.array(dxs), dys=np.array(dys), dthetas=np.array(dths),
                dx_range=rng(dxs), dy_range=rng(dys), dtheta_range=rng(dths),
                period=np.array(period), fps=np.array(fps),
                nb_steps_in_period=np.array(int(period * fps)))


class PolyReferenceMotion:
    """Host-side view of the baked table (same fields as the reference class).

    ``get_reference_motion`` here is a float64 numpy evaluation used by the host
    (e.g. ``reset`` bookkeeping); the hot path evaluates the table inside the env-step
    kernel.
    """

    def __init__(self, table_path: str):
        z = np.load(table_path, allow_pickle=False)
        self.data_array = z["coeffs"]
        self.dxs, self.dys, self.dthetas = list(z["dxs"]), list(z["dys"]), list(z["dthetas"])
        self.dx_range, self.dy_range, self.dtheta_range = list(z["dx_range"]), list(z["dy_range"]), list(
            z["dtheta_range"])
        self.period = float(z["period"])
        self.fps = float(z["fps"])
        self.nb_steps_in_period = int(z["nb_steps_in_period"])

    def vel_to_index(self, dx, dy, dtheta):
        dx = np.clip(dx, *self.dx_range)
        dy = np.clip(dy, *self.dy_range)
        dtheta = np.clip(dtheta, *self.dtheta_range)
        return (int(np.argmin(np.abs(np.array(self.dxs) - dx))), int(np.argmin(np.abs(np.array(self.dys) - dy))),
                int(np.argmin(np.abs(np.array(self.dthetas) - dtheta))))

    def get_reference_motion(self, dx, dy, dtheta, i):
        ix, iy, it = self.vel_to_index(dx, dy, dtheta)
        t = float(np.clip((i % self.nb_steps_in_period) / self.nb_steps_in_period, 0.0, 1.0))
        c = self.data_array[ix, iy, it]
        return np.polynomial.polynomial.polyval(t, c.T)
