"""Transpile a Python ``ODE(y, t, ps)`` right-hand side into a C++ device-function body
for the hipRTC path (``oe_model_compile``).

The reference hands the user's Python callable to odeint (ODElib/Framework.py:177-180,
:656).  The demo RHS functions (demo/Demo_InfectionStates.ipynb:60-128) are
straight-line arithmetic over ``y[i]`` and ``ps[i]``; this module translates that
subset:

* statements: assignments (also tuple unpacking ``a, b = ps[0], ps[1]`` / ``S, V = y``),
  augmented assignments, docstrings, one final ``return`` of ``np.array([...])``,
  a list or a tuple;
* expressions: ``+ - * / **``, unary ``-``/``+``, numeric constants, ``y[k]``/``ps[k]``
  with constant ``k``, ``t``, locals, numeric globals/closure constants, ``np.pi``/
  ``math.pi``/``math.e``, ``a if c else b`` with comparisons, and the math calls in
  ``_CALLS`` (numpy / math / builtins).

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
        ast.GtE: (">=", np.greater_equal)}


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

    # ---- expressions -> IR ----
    def index(self, node, length):
        if isinstance(node, ast.Constant) and isinstance(node.value, int) and not isinstance(node.value, bool):
            k = node.value
        elif isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub) and isinstance(node.operand, ast.Constant):
            k = -node.operand.value
        else:
            raise Unsupported("only constant integer indices into y / ps are supported")
        if k < 0:
            k += length
        if not (0 <= k < length):
            raise Unsupported(f"index {k} out of range (length {length})")
        return k

    def expr(self, n):
        if isinstance(n, ast.Constant):
            if isinstance(n.value, bool) or not isinstance(n.value, (int, float)):
                raise Unsupported(f"constant {n.value!r}")
            return ("const", float(n.value))
        if isinstance(n, ast.Name):
            if n.id in self.env:
                return ("var", n.id)
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

    def cond(self, n):
        if isinstance(n, ast.Compare) and len(n.ops) == 1 and type(n.ops[0]) in _CMP:
            return ("cmp", type(n.ops[0]), self.expr(n.left), self.expr(n.comparators[0]))
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
        for st in body:
            if self.outs is not None:
                raise Unsupported("statements after return")
            if isinstance(st, ast.Assign) and len(st.targets) == 1:
                tgt = st.targets[0]
                if isinstance(tgt, ast.Name):
                    self.assign([tgt.id], [self.expr(st.value)])
                elif isinstance(tgt, (ast.Tuple, ast.List)) and all(isinstance(e, ast.Name) for e in tgt.elts):
                    names = [e.id for e in tgt.elts]
                    self.assign(names, self.seq(st.value, len(names)))
                else:
                    raise Unsupported("assignment target")
            elif isinstance(st, ast.AugAssign) and isinstance(st.target, ast.Name) and st.target.id in self.env:
                op = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/"}.get(type(st.op))
                if op is None:
                    raise Unsupported("augmented operator")
                self.assign([st.target.id], [("bin", op, ("var", st.target.id), self.expr(st.value))])
            elif isinstance(st, ast.Return):
                self.outs = self.returned(st.value)
            elif isinstance(st, ast.Pass):
                continue
            else:
                raise Unsupported(type(st).__name__)
        if self.outs is None:
            raise Unsupported("no return")
        if len(self.outs) != self.S:
            raise Unsupported(f"returns {len(self.outs)} derivatives for {self.S} states")

    def assign(self, names, exprs):
        if len(names) == 1:
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
            self.stmts.append((name, ("var", tmp)))
            self.env.add(name)

    def returned(self, v):
        if isinstance(v, ast.Call) and isinstance(v.func, ast.Attribute) and isinstance(v.func.value, ast.Name) \
                and v.func.value.id in ("np", "numpy") and v.func.attr in ("array", "asarray") and len(v.args) == 1:
            v = v.args[0]
        if isinstance(v, (ast.List, ast.Tuple)):
            return [self.expr(e) for e in v.elts]
        raise Unsupported("return value must be np.array([...]), a list or a tuple")


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
    raise AssertionError(k)


def transpile(func, n_states: int, n_params: int) -> TranspiledRHS:
    tr = _Translator(func, n_states, n_params)
    tr.run()
    lines, declared = [], set()
    for name, expr in tr.stmts:
        if name in declared:
            lines.append(f"v_{name} = {_c(expr)};")
        else:
            lines.append(f"double v_{name} = {_c(expr)};")
            declared.add(name)
    for k, e in enumerate(tr.outs):
        lines.append(f"dy[{k}] = {_c(e)};")
    body = "\n".join("    " + ln for ln in lines)
    return TranspiledRHS(c_body=body, n_states=n_states, n_params=n_params, _stmts=tr.stmts, _outs=tr.outs)
