"""Transpile a Python ``ODE(y, t, ps)`` right-hand side into a C++ device-function body
for the hipRTC path (``oe_model_compile``).

The reference hands the user's Python callable to odeint (ODElib/Framework.py:177-180,
:656).  The demo RHS functions (demo/Demo_InfectionStates.ipynb:60-128) are
straight-line arithmetic over ``y[i]`` and ``ps[i]``; this module translates that
subset:

* statements: assignments (also tuple unpacking ``a, b = ps[0], ps[1]`` / ``S, V = y``),
  augmented assignments, docstrings, ``for i in range(...)`` loops with bounds known at
  translation time (unrolled), ``if``/``elif``/``else`` — on translation-time integers
  (loop variables, ``len()``) the branch is chosen while translating, on data both
  branches are evaluated and every variable / array element they assign is selected
  (``cond ? a : b``; no ``return`` inside such a branch) —, local arrays (``dy = np.zeros(len(y))`` /
  ``np.zeros_like(y)`` / ``np.empty(n)`` / ``[0.0] * n`` / a list literal) written and
  read element-wise (``dy[i] = ...``, ``dy[i] += ...``) or by slice (``dy[2:-2] = ...``,
  ``out[1:] += ...``, ``out *= ...``), one final ``return`` of ``np.array([...])``, a
  list, a tuple, a local array or an array expression;
* whole-array numpy arithmetic (``-k * y + np.exp(-y / 10.0) * t``, slices, broadcasting
  of scalars) is expanded element by element in numpy's operation order;
* expressions: ``+ - * / **``, unary ``-``/``+``, numeric constants, ``y[k]``/``ps[k]``/
  ``dy[k]`` with ``k`` an integer expression of constants, loop variables and ``len()``,
  ``t``, locals, numeric globals/closure constants, ``np.pi``/``math.pi``/``math.e``,
  ``a if c else b`` with comparisons, ``sum(...)`` / ``np.sum(...)`` of a slice or local
  array (expanded in numpy's summation order), and the math calls in ``_CALLS``
  (numpy / math / builtins).

Python evaluates ``a*b*c`` as ``(a*b)*c`` in IEEE double; the emitted C keeps every
parenthesisation and the library compiles with -ffp-contract=off, so each emitted
operation rounds exactly as the Python one does (transcendental calls are ~1 ulp).
Anything outside the subset raises ``Unsupported``.  The same intermediate form is also
evaluated with numpy (``TranspiledRHS.evaluate``) so ``models.resolve`` can check the
translation against the user's callable on probe points before compiling it.
"""
from __future__ import annotations

import ast
import inspect
import math
import textwrap
from dataclasses import dataclass

import numpy as np


class Unsupported(ValueError):
    """The callable uses Python outside the transpilable subset."""


# python call name -> (C function, numpy implementation, arity)
_CALLS = {
    "exp": ("exp", np.exp, 1), "log": ("log", np.log, 1), "sqrt": ("sqrt", np.sqrt, 1),
    "sin": ("sin", np.sin, 1), "cos": ("cos", np.cos, 1), "tan": ("tan", np.tan, 1),
    "tanh": ("tanh", np.tanh, 1), "sinh": ("sinh", np.sinh, 1), "cosh": ("cosh", np.cosh, 1),
    "arctan": ("atan", np.arctan, 1), "atan": ("atan", np.arctan, 1), "log10": ("log10", np.log10, 1),
    "log2": ("log2", np.log2, 1), "exp2": ("exp2", np.exp2, 1), "expm1": ("expm1", np.expm1, 1),
    "log1p": ("log1p", np.log1p, 1), "abs": ("fabs", np.abs, 1), "fabs": ("fabs", np.abs, 1),
    "absolute": ("fabs", np.abs, 1), "power": ("pow", np.power, 2), "pow": ("pow", np.power, 2),
    "maximum": ("fmax", np.fmax, 2), "minimum": ("fmin", np.fmin, 2), "max": ("fmax", np.fmax, 2),
    "min": ("fmin", np.fmin, 2), "fmax": ("fmax", np.fmax, 2), "fmin": ("fmin", np.fmin, 2),
}
_MODULES = {"np", "numpy", "math"}
_CMP = {ast.Lt: ("<", np.less), ast.LtE: ("<=", np.less_equal), ast.Gt: (">", np.greater),
        ast.GtE: (">=", np.greater_equal), ast.Eq: ("==", np.equal), ast.NotEq: ("!=", np.not_equal)}


def _c_float(x: float) -> str:
    if not math.isfinite(x):
        raise Unsupported("non-finite constant")
    return repr(float(x))


@dataclass
class TranspiledRHS:
    c_body: str
    n_states: int
    n_params: int
    _stmts: list
    _outs: list

    def evaluate(self, y, t, ps):
        """Evaluate the translated statements with numpy float64 (validation only)."""
        env = {}
        y = [np.float64(v) for v in y]
        ps = [np.float64(v) for v in ps]
        for name, expr in self._stmts:
            env[name] = _eval(expr, y, np.float64(t), ps, env)
        return np.array([_eval(e, y, np.float64(t), ps, env) for e in self._outs], dtype=float)


def _eval(e, y, t, ps, env):
    k = e[0]
    if k == "const":
        return np.float64(e[1])
    if k == "y":
        return y[e[1]]
    if k == "ps":
        return ps[e[1]]
    if k == "t":
        return t
    if k == "var":
        return env[e[1]]
    if k == "neg":
        return -_eval(e[1], y, t, ps, env)
    if k == "bin":
        a, b = _eval(e[2], y, t, ps, env), _eval(e[3], y, t, ps, env)
        with np.errstate(all="ignore"):
            op = e[1]
            if op == "+":
                return a + b
            if op == "-":
                return a - b
            if op == "*":
                return a * b
            if op == "/":
                return a / b
            if op == "sq":
                return a * a
            return np.power(a, b)
    if k == "call":
        args = [_eval(a, y, t, ps, env) for a in e[2]]
        with np.errstate(all="ignore"):
            return np.float64(_CALLS[e[1]][1](*args))
    if k == "ifexp":
        return _eval(e[2], y, t, ps, env) if _eval(e[1], y, t, ps, env) else _eval(e[3], y, t, ps, env)
    if k == "cmp":
        return bool(_CMP[e[1]][1](_eval(e[2], y, t, ps, env), _eval(e[3], y, t, ps, env)))
    if k == "and":
        return all(_eval(a, y, t, ps, env) for a in e[1])
    if k == "or":
        return any(_eval(a, y, t, ps, env) for a in e[1])
    if k == "not":
        return not _eval(e[1], y, t, ps, env)
    raise AssertionError(k)


class _Translator:
    def __init__(self, func, n_states, n_params):
        try:
            src = textwrap.dedent(inspect.getsource(func))
        except (OSError, TypeError) as exc:
            raise Unsupported(f"source of {func!r} is not available") from exc
        mod = ast.parse(src)
        fdefs = [n for n in mod.body if isinstance(n, ast.FunctionDef)]
        if not fdefs:
            raise Unsupported("not a plain `def` function")
        self.fdef = fdefs[0]
        args = [a.arg for a in self.fdef.args.args]
        if len(args) != 3 or self.fdef.args.vararg or self.fdef.args.kwarg:
            raise Unsupported("the RHS must be def f(y, t, ps)")
        self.yname, self.tname, self.pname = args
        self.S, self.P = int(n_states), int(n_params)
        cv = inspect.getclosurevars(func)
        self.consts = {}
        for name, val in list(cv.globals.items()) + list(cv.nonlocals.items()):
            if isinstance(val, (int, float, np.floating, np.integer)) and not isinstance(val, bool):
                self.consts[name] = float(val)
        self.env = set()
        self.stmts = []     # (name, expr-IR)
        self.outs = None
        self.ints = {}      # translation-time integers: loop variables, len(...), integer locals
        self.arrays = {}    # local arrays: name -> [element variable name or None (unset)]
        self.scopes = []    # branches of an `if` on data being translated: name -> fresh variable
        self.uid = 0
        self.constvals = {}  # float locals currently bound to a numeric literal (usable as indices)

    # ---- translation-time integers (indices, loop bounds) ----
    def length_of(self, name):
        if name == self.yname:
            return self.S
        if name == self.pname:
            return self.P
        if name in self.arrays:
            return len(self.arrays[name])
        raise Unsupported(f"len({name})")

    def intexpr(self, n):
        if isinstance(n, ast.Constant) and isinstance(n.value, int) and not isinstance(n.value, bool):
            return n.value
        if isinstance(n, ast.Name):
            if n.id in self.ints:
                return self.ints[n.id]
            if n.id in self.consts and float(self.consts[n.id]).is_integer() and n.id not in self.env:
                return int(self.consts[n.id])
            if n.id in self.constvals and float(self.constvals[n.id]).is_integer() and not self.scopes:
                return int(self.constvals[n.id])
            raise Unsupported(f"{n.id!r} is not an integer known at translation time")
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Name) and n.func.id == "len" and len(n.args) == 1 \
                and isinstance(n.args[0], ast.Name):
            return self.length_of(n.args[0].id)
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Name) and n.func.id == "int" and len(n.args) == 1:
            return self.intexpr(n.args[0])
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.USub):
            return -self.intexpr(n.operand)
        if isinstance(n, ast.BinOp):
            a, b = self.intexpr(n.left), self.intexpr(n.right)
            ops = {ast.Add: lambda: a + b, ast.Sub: lambda: a - b, ast.Mult: lambda: a * b,
                   ast.FloorDiv: lambda: a // b, ast.Mod: lambda: a % b}
            if type(n.op) in ops:
                return ops[type(n.op)]()
        raise Unsupported("integer expression")

    def int_sourced(self, n):
        """The expression derives from len() / int() / a translation-time integer (a bare
        numeric literal stays a float local, usable as an index while it holds it)."""
        for sub in ast.walk(n):
            if isinstance(sub, ast.Call) and isinstance(sub.func, ast.Name) and sub.func.id in ("len", "int"):
                return True
            if isinstance(sub, ast.Name) and sub.id in self.ints:
                return True
        return False

    def is_int(self, n):
        """True for an integer expression known at translation time (no y/ps/t data)."""
        if isinstance(n, ast.Constant) and isinstance(n.value, float):
            return False
        try:
            self.intexpr(n)
            return True
        except Unsupported:
            return False

    def index(self, node, length):
        k = self.intexpr(node)
        if k < 0:
            k += length
        if not (0 <= k < length):
            raise Unsupported(f"index {k} out of range (length {length})")
        return k

    def elements(self, n):
        """IR of the elements of y, ps, a local array, or a slice of one (for sum)."""
        if isinstance(n, ast.Name) and (n.id in (self.yname, self.pname) or n.id in self.arrays):
            base, sl = n.id, None
        elif isinstance(n, ast.Subscript) and isinstance(n.value, ast.Name) and isinstance(n.slice, ast.Slice):
            base, sl = n.value.id, n.slice
        else:
            raise Unsupported("sum() needs y, ps, a local array or a slice of one")
        length = self.length_of(base)
        idx = list(range(length))
        if sl is not None:
            lo = self.intexpr(sl.lower) if sl.lower is not None else None
            hi = self.intexpr(sl.upper) if sl.upper is not None else None
            st = self.intexpr(sl.step) if sl.step is not None else None
            idx = idx[slice(lo, hi, st)]
        return [self.element(base, k) for k in idx]

    def element(self, base, k):
        if base == self.yname:
            return ("y", k)
        if base == self.pname:
            return ("ps", k)
        var = self.arrays[base][k]
        if var is None:
            raise Unsupported(f"{base}[{k}] read before it is set")
        return ("var", var)

    def listexpr(self, n):
        """Scalar IR of a Python list built from literals, `+` concatenation and `*` repetition."""
        if isinstance(n, (ast.List, ast.Tuple)):
            return [self.expr(e) for e in n.elts]
        if isinstance(n, ast.BinOp) and isinstance(n.op, ast.Add):
            return self.listexpr(n.left) + self.listexpr(n.right)
        if isinstance(n, ast.BinOp) and isinstance(n.op, ast.Mult):
            if isinstance(n.left, (ast.List, ast.Tuple, ast.BinOp)) and self.is_int(n.right):
                return self.listexpr(n.left) * self.intexpr(n.right)
            if isinstance(n.right, (ast.List, ast.Tuple, ast.BinOp)) and self.is_int(n.left):
                return self.listexpr(n.right) * self.intexpr(n.left)
        raise Unsupported("list expression")

    # ---- whole-array (numpy elementwise) expressions -> list of scalar IR ----
    _BINOPS = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/"}

    def vexpr(self, n):
        """Elementwise IR of an array-valued expression (y, ps, a local array, a slice of
        one, or numpy arithmetic / ufunc calls involving them); None if `n` is scalar."""
        if isinstance(n, ast.Name):
            if n.id in (self.yname, self.pname) or n.id in self.arrays:
                return self.elements(n)
            return None
        if isinstance(n, ast.Subscript) and isinstance(n.slice, ast.Slice):
            return self.elements(n)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, (ast.USub, ast.UAdd)):
            v = self.vexpr(n.operand)
            if v is None or isinstance(n.op, ast.UAdd):
                return v
            return [("neg", e) for e in v]
        if isinstance(n, ast.BinOp) and (type(n.op) in self._BINOPS or isinstance(n.op, ast.Pow)):
            va, vb = self.vexpr(n.left), self.vexpr(n.right)
            if va is None and vb is None:
                return None
            if va is not None and vb is not None and len(va) != len(vb):
                raise Unsupported("array lengths differ")
            m = len(va if va is not None else vb)
            la = va if va is not None else [self.expr(n.left)] * m
            lb = vb if vb is not None else [self.expr(n.right)] * m
            if isinstance(n.op, ast.Pow):
                return [("bin", "sq", a, a) if b == ("const", 2.0) else ("bin", "pow", a, b) for a, b in zip(la, lb)]
            return [("bin", self._BINOPS[type(n.op)], a, b) for a, b in zip(la, lb)]
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute) and isinstance(n.func.value, ast.Name) \
                and n.func.value.id in ("np", "numpy"):
            if n.func.attr in ("array", "asarray") and len(n.args) == 1 and not n.keywords:
                a = n.args[0]
                if isinstance(a, (ast.List, ast.Tuple)) or (isinstance(a, ast.BinOp) and self.vexpr(a) is None):
                    return self.listexpr(a)
                return self.vexpr(a)
            if n.func.attr in _CALLS and not n.keywords:
                vs = [self.vexpr(a) for a in n.args]
                if all(v is None for v in vs):
                    return None
                m = {len(v) for v in vs if v is not None}
                if len(m) != 1 or len(n.args) != _CALLS[n.func.attr][2]:
                    raise Unsupported(f"np.{n.func.attr} arguments")
                m = m.pop()
                cols = [v if v is not None else [self.expr(a)] * m for v, a in zip(vs, n.args)]
                return [("call", n.func.attr, list(args)) for args in zip(*cols)]
        return None

    def expr(self, n):
        if isinstance(n, ast.Constant):
            if isinstance(n.value, bool) or not isinstance(n.value, (int, float)):
                raise Unsupported(f"constant {n.value!r}")
            return ("const", float(n.value))
        if isinstance(n, ast.Name):
            if n.id in self.arrays:
                raise Unsupported(f"array {n.id!r} used as a scalar")
            if self.defined(n.id):
                return ("var", self.lookup(n.id))
            if n.id in self.ints:
                return ("const", float(self.ints[n.id]))
            if n.id == self.tname:
                return ("t",)
            if n.id in self.consts:
                return ("const", self.consts[n.id])
            raise Unsupported(f"name {n.id!r}")
        if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name) and n.value.id in _MODULES:
            if n.attr == "pi":
                return ("const", math.pi)
            if n.attr == "e":
                return ("const", math.e)
            raise Unsupported(f"attribute {n.value.id}.{n.attr}")
        if isinstance(n, ast.Subscript) and isinstance(n.value, ast.Name):
            idx = n.slice.value if isinstance(n.slice, ast.Index) else n.slice  # py<3.9 compat
            if n.value.id == self.yname:
                return ("y", self.index(idx, self.S))
            if n.value.id == self.pname:
                return ("ps", self.index(idx, self.P))
            if n.value.id in self.arrays:
                return self.element(n.value.id, self.index(idx, len(self.arrays[n.value.id])))
            raise Unsupported(f"subscript of {n.value.id!r}")
        if isinstance(n, ast.UnaryOp):
            if isinstance(n.op, ast.USub):
                return ("neg", self.expr(n.operand))
            if isinstance(n.op, ast.UAdd):
                return self.expr(n.operand)
            raise Unsupported("unary operator")
        if isinstance(n, ast.BinOp):
            a, b = self.expr(n.left), self.expr(n.right)
            if isinstance(n.op, ast.Add):
                return ("bin", "+", a, b)
            if isinstance(n.op, ast.Sub):
                return ("bin", "-", a, b)
            if isinstance(n.op, ast.Mult):
                return ("bin", "*", a, b)
            if isinstance(n.op, ast.Div):
                return ("bin", "/", a, b)
            if isinstance(n.op, ast.Pow):
                if b == ("const", 2.0):
                    return ("bin", "sq", a, a)
                return ("bin", "pow", a, b)
            raise Unsupported("binary operator")
        if isinstance(n, ast.Call):
            f = n.func
            is_sum = (isinstance(f, ast.Name) and f.id == "sum") or (
                isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id in ("np", "numpy")
                and f.attr == "sum")
            if is_sum:
                if len(n.args) != 1 or n.keywords:
                    raise Unsupported("sum() of one sequence")
                return self.summation(self.elements(n.args[0]), pairwise=not isinstance(f, ast.Name))
            if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id in _MODULES:
                name = f.attr
            elif isinstance(f, ast.Name) and f.id in ("abs", "max", "min", "pow"):
                name = f.id
            else:
                raise Unsupported("call")
            if name not in _CALLS or n.keywords:
                raise Unsupported(f"call {name}")
            cfun, _, arity = _CALLS[name]
            if len(n.args) != arity:
                raise Unsupported(f"{name} with {len(n.args)} arguments")
            return ("call", name, [self.expr(a) for a in n.args])
        if isinstance(n, ast.IfExp):
            return ("ifexp", self.cond(n.test), self.expr(n.body), self.expr(n.orelse))
        raise Unsupported(type(n).__name__)

    @staticmethod
    def summation(xs, pairwise):
        """Python's sum() adds left to right from 0; numpy's add.reduce (pairwise_sum)
        does the same below 8 elements and otherwise runs 8 strided accumulators,
        combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the remainder."""
        if not xs:
            return ("const", 0.0)
        if not pairwise or len(xs) < 8:
            acc = xs[0]  # 0 + x0 == x0
            for x in xs[1:]:
                acc = ("bin", "+", acc, x)
            return acc
        if len(xs) > 128:
            raise Unsupported("np.sum of more than 128 elements")
        r = list(xs[:8])
        m = len(xs) - len(xs) % 8
        for i in range(8, m, 8):
            for j in range(8):
                r[j] = ("bin", "+", r[j], xs[i + j])
        acc = ("bin", "+", ("bin", "+", ("bin", "+", r[0], r[1]), ("bin", "+", r[2], r[3])),
               ("bin", "+", ("bin", "+", r[4], r[5]), ("bin", "+", r[6], r[7])))
        for x in xs[m:]:
            acc = ("bin", "+", acc, x)
        return acc

    def cond(self, n):
        if isinstance(n, ast.Compare) and all(type(o) in _CMP for o in n.ops):
            terms = [self.expr(n.left)] + [self.expr(c) for c in n.comparators]
            parts = [("cmp", type(o), a, b) for o, a, b in zip(n.ops, terms, terms[1:])]
            return parts[0] if len(parts) == 1 else ("and", parts)
        if isinstance(n, ast.BoolOp):
            return ("and" if isinstance(n.op, ast.And) else "or", [self.cond(v) for v in n.values])
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.Not):
            return ("not", self.cond(n.operand))
        raise Unsupported("condition")

    def seq(self, node, n_targets):
        """Right-hand side of a tuple assignment -> list of IR."""
        if isinstance(node, (ast.Tuple, ast.List)):
            if len(node.elts) != n_targets:
                raise Unsupported("unpacking length mismatch")
            return [self.expr(e) for e in node.elts]
        if isinstance(node, ast.Name) and node.id in (self.yname, self.pname):
            length = self.S if node.id == self.yname else self.P
            if n_targets != length:
                raise Unsupported(f"unpacking {node.id} needs {length} names")
            kind = "y" if node.id == self.yname else "ps"
            return [(kind, k) for k in range(length)]
        raise Unsupported("tuple assignment source")

    # ---- statements ----
    def run(self):
        body = list(self.fdef.body)
        if body and isinstance(body[0], ast.Expr) and isinstance(body[0].value, ast.Constant) \
                and isinstance(body[0].value.value, str):
            body = body[1:]
        self.block(body)
        if self.outs is None:
            raise Unsupported("no return")
        if len(self.outs) != self.S:
            raise Unsupported(f"returns {len(self.outs)} derivatives for {self.S} states")

    _AUG = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/"}

    def block(self, body):
        for st in body:
            if self.outs is not None:
                raise Unsupported("statements after return")
            if isinstance(st, ast.Assign) and len(st.targets) == 1:
                tgt = st.targets[0]
                if isinstance(tgt, ast.Name):
                    arr = self.array_value(st.value)
                    if arr is not None:
                        self.new_array(tgt.id, arr)
                    elif tgt.id in self.arrays:
                        raise Unsupported(f"array {tgt.id!r} reassigned")
                    elif tgt.id not in self.env and not self.scopes and self.is_int(st.value) \
                            and self.int_sourced(st.value):
                        self.ints[tgt.id] = self.intexpr(st.value)  # e.g. n = len(y), j = i + 1
                    else:
                        self.ints.pop(tgt.id, None)
                        self.assign([tgt.id], [self.expr(st.value)])
                elif isinstance(tgt, ast.Subscript) and isinstance(tgt.value, ast.Name) and tgt.value.id in self.arrays:
                    if isinstance(tgt.slice, ast.Slice):
                        self.set_slice(tgt, lambda old, new: new, st.value)
                    else:
                        self.set_element(tgt, self.expr(st.value))
                elif isinstance(tgt, (ast.Tuple, ast.List)) and all(isinstance(e, ast.Name) for e in tgt.elts):
                    names = [e.id for e in tgt.elts]
                    self.assign(names, self.seq(st.value, len(names)))
                else:
                    raise Unsupported("assignment target")
            elif isinstance(st, ast.AugAssign) and type(st.op) in self._AUG:
                op = self._AUG[type(st.op)]
                if isinstance(st.target, ast.Name) and st.target.id in self.ints and self.is_int(st.value) \
                        and op in "+-*":
                    a, b = self.ints[st.target.id], self.intexpr(st.value)
                    self.ints[st.target.id] = a + b if op == "+" else a - b if op == "-" else a * b
                elif isinstance(st.target, ast.Name) and st.target.id in self.ints:
                    old = ("const", float(self.ints.pop(st.target.id)))
                    self.assign([st.target.id], [("bin", op, old, self.expr(st.value))])
                elif isinstance(st.target, ast.Name) and self.defined(st.target.id) and st.target.id not in self.arrays:
                    self.assign([st.target.id], [("bin", op, ("var", self.lookup(st.target.id)), self.expr(st.value))])
                elif isinstance(st.target, ast.Subscript) and isinstance(st.target.value, ast.Name) \
                        and st.target.value.id in self.arrays and isinstance(st.target.slice, ast.Slice):
                    self.set_slice(st.target, lambda old, new, op=op: ("bin", op, old, new), st.value)
                elif isinstance(st.target, ast.Subscript) and isinstance(st.target.value, ast.Name) \
                        and st.target.value.id in self.arrays:
                    old = self.expr(st.target)
                    self.set_element(st.target, ("bin", op, old, self.expr(st.value)))
                elif isinstance(st.target, ast.Name) and st.target.id in self.arrays:
                    whole = ast.Subscript(value=ast.Name(id=st.target.id, ctx=ast.Load()),
                                          slice=ast.Slice(lower=None, upper=None, step=None), ctx=ast.Store())
                    self.set_slice(whole, lambda old, new, op=op: ("bin", op, old, new), st.value)
                else:
                    raise Unsupported("augmented assignment target")
            elif isinstance(st, ast.For):
                self.unroll(st)
            elif isinstance(st, ast.If):
                # a condition on translation-time integers (loop variables, len()) picks one
                # branch while translating; a condition on data evaluates both branches
                # and selects every variable / element either branch assigns
                try:
                    static = self.static_cond(st.test)
                except Unsupported:
                    static = None
                if static is None:
                    self.data_if(st)
                else:
                    self.block(st.body if static else st.orelse)
            elif isinstance(st, ast.Return):
                self.outs = self.returned(st.value)
            elif isinstance(st, ast.Pass):
                continue
            else:
                raise Unsupported(type(st).__name__)

    _ICMP = {ast.Eq: lambda a, b: a == b, ast.NotEq: lambda a, b: a != b, ast.Lt: lambda a, b: a < b,
             ast.LtE: lambda a, b: a <= b, ast.Gt: lambda a, b: a > b, ast.GtE: lambda a, b: a >= b}

    def defined(self, name):
        return name in self.env or any(name in d for d in self.scopes)

    def lookup(self, name):
        for d in reversed(self.scopes):
            if name in d:
                return d[name]
        return name

    def data_if(self, st):
        cond = self.cond(st.test)
        before_arrays = {k: list(v) for k, v in self.arrays.items()}
        before_ints = dict(self.ints)
        results = []
        for body in (st.body, st.orelse):
            self.arrays = {k: list(v) for k, v in before_arrays.items()}
            self.scopes.append({})
            self.block(body)
            names = self.scopes.pop()
            if self.outs is not None:
                raise Unsupported("return inside an `if` on data")
            if self.ints != before_ints or set(self.arrays) != set(before_arrays):
                raise Unsupported("an `if` on data may only assign floats and array elements")
            results.append((names, self.arrays))
        (tn, ta), (en, ea) = results
        self.arrays = {k: list(v) for k, v in before_arrays.items()}
        for name in sorted(set(tn) | set(en)):
            if (name not in tn or name not in en) and not self.defined(name):
                raise Unsupported(f"{name!r} is assigned in only one branch of an `if` on data")
            a = tn.get(name, self.lookup(name))
            b = en.get(name, self.lookup(name))
            self.assign([name], [("ifexp", cond, ("var", a), ("var", b))])
        for arr, elems in before_arrays.items():
            for k, orig in enumerate(elems):
                a, b = ta[arr][k], ea[arr][k]
                if a == orig and b == orig:
                    continue
                if a is None or b is None:
                    raise Unsupported(f"{arr}[{k}] is set in only one branch of an `if` on data")
                self.arrays[arr][k] = self.bind(f"{arr}__{k}", ("ifexp", cond, ("var", a), ("var", b)))

    def static_cond(self, n):
        if isinstance(n, ast.Compare) and all(type(o) in self._ICMP for o in n.ops):
            vals = [self.intexpr(n.left)] + [self.intexpr(c) for c in n.comparators]
            return all(self._ICMP[type(o)](a, b) for o, a, b in zip(n.ops, vals, vals[1:]))
        if isinstance(n, ast.BoolOp):
            parts = [self.static_cond(v) for v in n.values]
            return all(parts) if isinstance(n.op, ast.And) else any(parts)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.Not):
            return not self.static_cond(n.operand)
        if isinstance(n, ast.Constant) and isinstance(n.value, bool):
            return n.value
        raise Unsupported("`if` on data (only conditions on loop variables / len() / integer constants)")

    def unroll(self, st):
        it = st.iter
        if not (isinstance(st.target, ast.Name) and isinstance(it, ast.Call) and isinstance(it.func, ast.Name)
                and it.func.id == "range" and 1 <= len(it.args) <= 3 and not it.keywords and not st.orelse):
            raise Unsupported("only `for i in range(...)` loops with known bounds")
        bounds = [self.intexpr(a) for a in it.args]
        values = range(*bounds)
        if len(values) > 4096:
            raise Unsupported("loop longer than 4096 iterations")
        name = st.target.id
        if name in self.env or name in self.arrays:
            raise Unsupported(f"loop variable {name!r} shadows a local")
        for v in values:
            self.ints[name] = v
            self.block(st.body)
            if self.outs is not None:
                raise Unsupported("return inside a loop")

    def array_value(self, v):
        """Element IR list if `v` constructs a local array, else None."""
        def length(arg):
            return self.length_of(arg.id) if isinstance(arg, ast.Name) and (
                arg.id in (self.yname, self.pname) or arg.id in self.arrays) else None
        if isinstance(v, ast.Call) and isinstance(v.func, ast.Attribute) and isinstance(v.func.value, ast.Name) \
                and v.func.value.id in ("np", "numpy") and len(v.args) == 1:
            attr, arg = v.func.attr, v.args[0]
            if attr in ("zeros", "empty"):
                n = self.intexpr(arg)
                return [("const", 0.0) if attr == "zeros" else None] * n
            if attr in ("zeros_like", "empty_like"):
                n = length(arg)
                if n is None:
                    raise Unsupported(f"np.{attr} of a non-array")
                return [("const", 0.0) if attr == "zeros_like" else None] * n
            return self.vexpr(v)  # np.array(...) / np.asarray(...) / elementwise ufuncs
        if isinstance(v, ast.List) or (isinstance(v, ast.BinOp) and (
                isinstance(v.left, (ast.List, ast.Tuple)) or isinstance(v.right, (ast.List, ast.Tuple)))):
            return self.listexpr(v)
        return self.vexpr(v)

    def new_array(self, name, elems):
        if name in self.env or name in (self.yname, self.pname, self.tname):
            raise Unsupported(f"array {name!r} shadows a scalar or an argument")
        self.arrays[name] = [None] * len(elems)
        for k, e in enumerate(elems):
            if e is not None:
                self.arrays[name][k] = self.bind(f"{name}__{k}", e)

    def set_slice(self, tgt, combine, value):
        """arr[a:b:c] = value / arr[a:b:c] op= value, elementwise (value broadcast if scalar)."""
        name = tgt.value.id
        sl = tgt.slice
        idx = list(range(len(self.arrays[name])))[slice(
            self.intexpr(sl.lower) if sl.lower is not None else None,
            self.intexpr(sl.upper) if sl.upper is not None else None,
            self.intexpr(sl.step) if sl.step is not None else None)]
        vec = self.vexpr(value)
        if vec is None:
            vec = [self.expr(value)] * len(idx)
        if len(vec) != len(idx):
            raise Unsupported("slice assignment length mismatch")
        olds = [self.element(name, k) if self.arrays[name][k] is not None else None for k in idx]
        news = [combine(o, v) if o is not None or combine(("const", 0.0), v) == v else None
                for o, v in zip(olds, vec)]
        if any(nv is None for nv in news):
            raise Unsupported(f"{name}[...] updated before it is set")
        for k, nv in zip(idx, news):  # all right-hand sides read before any element is written
            self.arrays[name][k] = self.bind(f"{name}__{k}", nv)

    def set_element(self, tgt, e):
        name = tgt.value.id
        k = self.index(tgt.slice, len(self.arrays[name]))
        self.arrays[name][k] = self.bind(f"{name}__{k}", e)

    def bind(self, var, e):
        if self.scopes:  # inside a branch of an `if` on data: never overwrite a live value
            var = f"{var}__b{self.uid}"
            self.uid += 1
        self.stmts.append((var, e))
        self.env.add(var)
        return var

    def assign(self, names, exprs):
        if len(names) == 1:
            if exprs[0][0] == "const" and not self.scopes:
                self.constvals[names[0]] = exprs[0][1]
            else:
                self.constvals.pop(names[0], None)
            if self.scopes:
                self.scopes[-1][names[0]] = self.bind(names[0], exprs[0])
                return
            self.stmts.append((names[0], exprs[0]))
            self.env.add(names[0])
            return
        tmps = []
        for k, e in enumerate(exprs):  # simultaneous assignment semantics
            tmp = f"__tup{len(self.stmts)}_{k}"
            self.stmts.append((tmp, e))
            self.env.add(tmp)
            tmps.append(tmp)
        for name, tmp in zip(names, tmps):
            self.assign([name], [("var", tmp)])

    def returned(self, v):
        if isinstance(v, ast.Call) and isinstance(v.func, ast.Attribute) and isinstance(v.func.value, ast.Name) \
                and v.func.value.id in ("np", "numpy") and v.func.attr in ("array", "asarray") and len(v.args) == 1:
            v = v.args[0]
        if isinstance(v, (ast.List, ast.Tuple)):
            return [self.expr(e) for e in v.elts]
        if isinstance(v, ast.BinOp) and (isinstance(v.left, (ast.List, ast.Tuple))
                                         or isinstance(v.right, (ast.List, ast.Tuple))):
            return self.listexpr(v)
        vec = self.vexpr(v)
        if vec is not None:
            return vec
        raise Unsupported("return value must be np.array([...]), a list, a tuple or an array expression")


def _c(e) -> str:
    k = e[0]
    if k == "const":
        return _c_float(e[1])
    if k == "y":
        return f"y[{e[1]}]"
    if k == "ps":
        return f"ps[{e[1]}]"
    if k == "t":
        return "t"
    if k == "var":
        return "v_" + e[1]
    if k == "neg":
        return f"(-{_c(e[1])})"
    if k == "bin":
        if e[1] == "sq":
            a = _c(e[2])
            return f"({a} * {a})"
        if e[1] == "pow":
            return f"pow({_c(e[2])}, {_c(e[3])})"
        return f"({_c(e[2])} {e[1]} {_c(e[3])})"
    if k == "call":
        return f"{_CALLS[e[1]][0]}(" + ", ".join(_c(a) for a in e[2]) + ")"
    if k == "ifexp":
        return f"({_c(e[1])} ? {_c(e[2])} : {_c(e[3])})"
    if k == "cmp":
        return f"({_c(e[2])} {_CMP[e[1]][0]} {_c(e[3])})"
    if k in ("and", "or"):
        return "(" + (" && " if k == "and" else " || ").join(_c(a) for a in e[1]) + ")"
    if k == "not":
        return f"(!{_c(e[1])})"
    raise AssertionError(k)


_POLY_MAX_TERMS = 4096


def _padd(a, b, sign=1):
    out = dict(a)
    for m, c in b.items():
        v = out.get(m, 0) + sign * c
        if v:
            out[m] = v
        else:
            out.pop(m, None)
    return out


def _pmul(a, b):
    out = {}
    for ma, ca in a.items():
        for mb, cb in b.items():
            exps = dict(ma)
            for v, e in mb:
                exps[v] = exps.get(v, 0) + e
            m = tuple(sorted(exps.items()))
            c = out.get(m, 0) + ca * cb
            if c:
                out[m] = c
            else:
                out.pop(m, None)
    if len(out) > _POLY_MAX_TERMS:
        raise _NotPolynomial
    return out


class _NotPolynomial(Exception):
    pass


def _poly(e, env):
    """Expression -> {monomial: exact rational coefficient}; monomial = sorted
    ((('y'|'p'), index), exponent) pairs.  Raises _NotPolynomial for t, calls, branches,
    comparisons and division by anything but a non-zero constant."""
    from fractions import Fraction
    k = e[0]
    if k == "const":
        c = Fraction(float(e[1]))
        return {(): c} if c else {}
    if k in ("y", "ps"):
        return {((("y" if k == "y" else "p", e[1]), 1),): Fraction(1)}
    if k == "var":
        return env[e[1]]
    if k == "neg":
        return {m: -c for m, c in _poly(e[1], env).items()}
    if k == "bin":
        op = e[1]
        a = _poly(e[2], env)
        if op == "sq":
            return _pmul(a, a)
        b = _poly(e[3], env)
        if op == "+":
            return _padd(a, b)
        if op == "-":
            return _padd(a, b, -1)
        if op == "*":
            return _pmul(a, b)
        if op == "/":
            if set(b) != {()}:
                raise _NotPolynomial
            return {m: c / b[()] for m, c in a.items()}
        if op == "pow":
            if set(b) - {()}:
                raise _NotPolynomial
            n = b.get((), 0)
            if n.denominator != 1 or not 0 <= n <= 8:
                raise _NotPolynomial
            out = {(): Fraction(1)}
            for _ in range(int(n)):
                out = _pmul(out, a)
            return out
    raise _NotPolynomial


def polynomial_form(tr: "TranspiledRHS"):
    """Exact algebraic normal form of a transpiled RHS: one {monomial: rational
    coefficient} per dy[k], or None when the RHS is not a polynomial in y and ps with
    constant coefficients (it reads t, calls a function, branches on data, or divides by
    a non-constant).  Two right-hand sides with equal forms compute the same
    mathematical function; they can differ only in floating-point rounding order."""
    env = {}
    try:
        for name, expr in tr._stmts:
            env[name] = _poly(expr, env)
        return tuple(tuple(sorted(_poly(e, env).items())) for e in tr._outs)
    except _NotPolynomial:
        return None


def transpile(func, n_states: int, n_params: int) -> TranspiledRHS:
    tr = _Translator(func, n_states, n_params)
    tr.run()
    lines, declared = [], set()
    for name, expr in tr.stmts:
        if name in declared:
            lines.append(f"v_{name} = {_c(expr)};")
        else:
            lines.append(f"R v_{name} = {_c(expr)};")  # R: double, or a dual number for the Jacobian
            declared.add(name)
    for k, e in enumerate(tr.outs):
        lines.append(f"dy[{k}] = {_c(e)};")
    body = "\n".join("    " + ln for ln in lines)
    return TranspiledRHS(c_body=body, n_states=n_states, n_params=n_params, _stmts=tr.stmts, _outs=tr.outs)
