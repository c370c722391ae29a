"""A small WGSL interpreter for the compute shader of the reference (test infrastructure).

The reference's hot path is WGSL (`assets/compute_shader.wgsl`) run by wgpu, and neither
wgpu, naga nor a Vulkan driver exists in this image.  This module parses and executes that
WGSL source itself, so the golden fixtures of `tests/golden/make_wgsl_golden.py` are outputs
of the reference's own shader code rather than of our restatement (oracle/rps_oracle.c).

Scope: the WGSL subset that file uses -- structs, storage / uniform / private globals,
consts, functions, let/var, if/else, for, break/continue/return, vector and struct values,
and the builtins abs, dot, clamp, mix, sqrt, min, max, arrayLength and the scalar / vector
constructors and conversions.

Arithmetic (the points that fix results bit for bit):
  * f32 ops are IEEE single precision, each rounded (numpy float32 scalars), no FMA
    contraction; sqrt is correctly rounded.  i32/u32 wrap modulo 2^32.
  * Abstract literals are folded exactly (Python int / float) and converted to the concrete
    type of the other operand, as WGSL's abstract numerics specify.
  * i32(f32) truncates toward zero and saturates; NaN converts to 0 (WGSL leaves NaN
    conversion to the implementation; this is the choice DESIGN.md §3.1 documents).
  * mix(a, b, t) = a * (1 - t) + b * t; clamp(x, lo, hi) keeps NaN (x < lo -> lo,
    x > hi -> hi); max/min pick the other operand when one is NaN.
Dispatch semantics (`Dispatch`): WGSL leaves the shader's intra-dispatch races undefined
(pre_simulation_step writes predicted_positions that other invocations read; simulation_step
writes velocities that other invocations read).  Two schedules are offered:
  * "isolated": each invocation sees the buffers as they were at the dispatch start plus its
    own writes; all writes land when the dispatch ends.
  * "lockstep": the entry function's top-level statements run one at a time across all
    invocations, each statement's writes landing before the next statement runs.
Two invocations writing the same element in one step is reported as an error (a race the
schedules above do not define).
"""
from __future__ import annotations

import copy
import re
import warnings

import numpy as np

F32, I32, U32 = np.float32, np.int32, np.uint32
warnings.filterwarnings("ignore", category=RuntimeWarning)

# ---------------------------------------------------------------------------------------
# Lexer
# ---------------------------------------------------------------------------------------
TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<num>0[xX][0-9a-fA-F]+[iu]?|[0-9]+\.[0-9]*(?:[eE][+-]?[0-9]+)?[fh]?|\.[0-9]+(?:[eE][+-]?[0-9]+)?[fh]?|[0-9]+(?:[eE][+-]?[0-9]+)[fh]?|[0-9]+[iuf]?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>->|\+\+|--|\+=|-=|\*=|/=|%=|&=|\|=|==|!=|<=|>=|&&|\|\||<<|>>|[-+*/%<>=!&|^~(){}\[\];:,.@])
""", re.S | re.X)


def tokenize(src):
    out, pos = [], 0
    while pos < len(src):
        m = TOKEN_RE.match(src, pos)
        if not m:
            raise SyntaxError(f"bad character at {src[pos:pos + 20]!r}")
        pos = m.end()
        if m.lastgroup != "ws":
            out.append((m.lastgroup, m.group()))
    out.append(("eof", ""))
    return out


# ---------------------------------------------------------------------------------------
# Parser -> tuples
# ---------------------------------------------------------------------------------------
class Parser:
    def __init__(self, src):
        self.t = tokenize(src)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k][1]

    def kind(self, k=0):
        return self.t[self.i + k][0]

    def take(self, want=None):
        tok = self.t[self.i][1]
        if want is not None and tok != want:
            raise SyntaxError(f"expected {want!r}, got {tok!r} near token {self.i}")
        self.i += 1
        return tok

    def accept(self, want):
        if self.peek() == want:
            self.i += 1
            return True
        return False

    # -- types --
    def type_(self):
        name = self.take()
        if self.accept("<"):
            args = [self.type_or_expr()]
            while self.accept(","):
                args.append(self.type_or_expr())
            self.close_angle()
            return (name, tuple(args))
        return (name, ())

    def type_or_expr(self):
        if self.kind() == "num":
            return ("lit", self.take())
        if self.kind() == "id" and self.peek() in ("read_write", "read", "storage", "uniform", "private",
                                                  "function", "workgroup"):
            return ("as", self.take())
        return self.type_()

    def close_angle(self):
        if self.peek() == ">>":  # split '>>' closing two template lists
            self.t[self.i] = ("op", ">")
            self.t.insert(self.i + 1, ("op", ">"))
        self.take(">")

    def attributes(self):
        attrs = []
        while self.accept("@"):
            name = self.take()
            args = []
            if self.accept("("):
                while not self.accept(")"):
                    args.append(self.take())
            attrs.append((name, args))
        return attrs

    # -- top level --
    def module(self):
        decls = []
        while self.kind() != "eof":
            attrs = self.attributes()
            kw = self.peek()
            if kw == "struct":
                self.take()
                name = self.take()
                self.take("{")
                fields = []
                while not self.accept("}"):
                    self.attributes()
                    fname = self.take()
                    self.take(":")
                    fields.append((fname, self.type_()))
                    self.accept(",")
                decls.append(("struct", name, fields))
                self.accept(";")
            elif kw == "var":
                self.take()
                space = None
                if self.accept("<"):
                    space = [self.take()]
                    while self.accept(","):
                        space.append(self.take())
                    self.close_angle()
                name = self.take()
                self.take(":")
                ty = self.type_()
                init = self.expr() if self.accept("=") else None
                self.take(";")
                decls.append(("var", name, space, ty, init, attrs))
            elif kw == "const":
                self.take()
                name = self.take()
                ty = self.type_() if self.accept(":") else None
                self.take("=")
                init = self.expr()
                self.take(";")
                decls.append(("const", name, ty, init))
            elif kw == "fn":
                self.take()
                name = self.take()
                self.take("(")
                params = []
                while not self.accept(")"):
                    self.attributes()
                    pname = self.take()
                    self.take(":")
                    params.append((pname, self.type_()))
                    self.accept(",")
                ret = None
                if self.accept("->"):
                    self.attributes()
                    ret = self.type_()
                body = self.block()
                decls.append(("fn", name, params, ret, body, attrs))
            else:
                raise SyntaxError(f"unexpected {kw!r} at top level")
        return decls

    # -- statements --
    def block(self):
        self.take("{")
        stmts = []
        while not self.accept("}"):
            stmts.append(self.stmt())
        return ("block", stmts)

    def stmt(self, need_semi=True):
        p = self.peek()
        if p == "{":
            return self.block()
        if p in ("let", "var", "const"):
            self.take()
            name = self.take()
            ty = self.type_() if self.accept(":") else None
            init = self.expr() if self.accept("=") else None
            if need_semi:
                self.take(";")
            return ("decl", p, name, ty, init)
        if p == "if":
            self.take()
            cond = self.expr()
            then = self.block()
            other = None
            if self.accept("else"):
                other = self.stmt() if self.peek() == "if" else self.block()
            return ("if", cond, then, other)
        if p == "for":
            self.take()
            self.take("(")
            init = None if self.peek() == ";" else self.stmt(need_semi=False)
            self.take(";")
            cond = None if self.peek() == ";" else self.expr()
            self.take(";")
            upd = None if self.peek() == ")" else self.stmt(need_semi=False)
            self.take(")")
            body = self.block()
            return ("for", init, cond, upd, body)
        if p in ("break", "continue"):
            self.take()
            self.take(";")
            return (p,)
        if p == "return":
            self.take()
            val = None if self.peek() == ";" else self.expr()
            self.take(";")
            return ("return", val)
        # assignment / increment / call
        lhs = self.expr()
        op = self.peek()
        if op in ("=", "+=", "-=", "*=", "/=", "%=", "&=", "|="):
            self.take()
            rhs = self.expr()
            st = ("assign", op, lhs, rhs)
        elif op in ("++", "--"):
            self.take()
            st = ("assign", "+=" if op == "++" else "-=", lhs, ("lit", "1"))
        else:
            st = ("expr", lhs)
        if need_semi:
            self.take(";")
        return st

    # -- expressions (precedence climbing) --
    BIN = [("||",), ("&&",), ("|",), ("^",), ("&",), ("==", "!="), ("<", ">", "<=", ">="), ("<<", ">>"),
           ("+", "-"), ("*", "/", "%")]

    def expr(self, level=0):
        if level == len(self.BIN):
            return self.unary()
        lhs = self.expr(level + 1)
        while self.peek() in self.BIN[level]:
            op = self.take()
            rhs = self.expr(level + 1)
            lhs = ("bin", op, lhs, rhs)
        return lhs

    def unary(self):
        p = self.peek()
        if p in ("-", "!", "~", "&", "*"):
            self.take()
            return ("un", p, self.unary())
        return self.postfix(self.primary())

    def primary(self):
        k, p = self.t[self.i]
        if p == "(":
            self.take()
            e = self.expr()
            self.take(")")
            return e
        if k == "num":
            self.take()
            return ("lit", p)
        if p in ("true", "false"):
            self.take()
            return ("bool", p == "true")
        if k == "id":
            name = self.take()
            targs = ()
            if self.peek() == "<" and name in ("vec2", "vec3", "vec4", "array", "mat4x4"):
                self.take("<")
                targs = [self.type_or_expr()]
                while self.accept(","):
                    targs.append(self.type_or_expr())
                self.close_angle()
                targs = tuple(targs)
            if self.accept("("):
                args = []
                while not self.accept(")"):
                    args.append(self.expr())
                    self.accept(",")
                return ("call", name, targs, args)
            return ("id", name)
        raise SyntaxError(f"unexpected {p!r}")

    def postfix(self, e):
        while True:
            if self.accept("."):
                e = ("member", e, self.take())
            elif self.accept("["):
                idx = self.expr()
                self.take("]")
                e = ("index", e, idx)
            else:
                return e


# ---------------------------------------------------------------------------------------
# Values
# ---------------------------------------------------------------------------------------
SCALAR = {"f32": F32, "i32": I32, "u32": U32}


class Abstract:
    """Abstract numeric literal (exact until it meets a concrete type)."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v


def lit(s):
    s = s.lower()
    if s.startswith("0x"):
        if s.endswith("u"):
            return U32(int(s[:-1], 16))
        if s.endswith("i"):
            return I32(int(s[:-1], 16))
        return Abstract(int(s, 16))
    if s.endswith("u"):
        return U32(int(s[:-1]))
    if s.endswith("i"):
        return I32(int(s[:-1]))
    if s.endswith("f"):
        return F32(float(s[:-1]))
    if any(c in s for c in ".e"):
        return Abstract(float(s))
    return Abstract(int(s))


def concretize(v, like):
    """Convert an abstract value to the scalar type of `like` (a scalar or an array)."""
    if not isinstance(v, Abstract):
        return v
    if isinstance(like, np.ndarray):
        t = like.dtype.type
    elif isinstance(like, Abstract):
        return v
    else:
        t = type(like)
    return t(v.v)


def default_concrete(v):
    if isinstance(v, Abstract):
        return F32(v.v) if isinstance(v.v, float) else I32(v.v)
    return v


def is_vec(v):
    return isinstance(v, np.ndarray)


def binop(op, a, b):
    if isinstance(a, Abstract) and isinstance(b, Abstract):
        x, y = a.v, b.v
        if op == "/" and isinstance(x, int) and isinstance(y, int):
            return Abstract(int(x / y))
        return Abstract({"+": lambda: x + y, "-": lambda: x - y, "*": lambda: x * y, "/": lambda: x / y,
                         "%": lambda: x % y}[op]()) if op in "+-*/%" else compare(op, x, y)
    a = concretize(a, b)
    b = concretize(b, a)
    if op in ("==", "!=", "<", ">", "<=", ">="):
        return compare(op, a, b)
    if op in ("&&", "||"):
        return bool(a) and bool(b) if op == "&&" else bool(a) or bool(b)
    kind = (a.dtype if is_vec(a) else np.dtype(type(a))).kind
    if kind == "f":
        r = {"+": np.add, "-": np.subtract, "*": np.multiply, "/": np.divide}[op](a, b)
        return r.astype(F32) if is_vec(r) else F32(r)
    # integers: wrap modulo 2^32
    t = (a.dtype if is_vec(a) else np.dtype(type(a))).type
    x, y = np.asarray(a, dtype=np.int64), np.asarray(b, dtype=np.int64)
    if op == "+":
        r = x + y
    elif op == "-":
        r = x - y
    elif op == "*":
        r = x * y
    elif op == "/":
        r = np.trunc(x / y).astype(np.int64)
    elif op == "%":
        r = np.fmod(x, y)
    elif op == "&":
        r = x & y
    elif op == "|":
        r = x | y
    elif op == "^":
        r = x ^ y
    elif op == "<<":
        r = x << (y & 31)
    elif op == ">>":
        r = x >> (y & 31)
    else:
        raise ValueError(op)
    r = (r & 0xFFFFFFFF).astype(np.uint32).view(t) if t is I32 else (r & 0xFFFFFFFF).astype(np.uint32)
    return r if is_vec(a) or is_vec(b) else t(r)


def compare(op, a, b):
    f = {"==": np.equal, "!=": np.not_equal, "<": np.less, ">": np.greater, "<=": np.less_equal,
         ">=": np.greater_equal}[op]
    r = f(a, b)
    return bool(r) if np.ndim(r) == 0 else r


def convert(t, v):
    """Value conversion to scalar type t (WGSL i32(x), u32(x), f32(x))."""
    v = default_concrete(v) if not isinstance(v, Abstract) else v
    if isinstance(v, Abstract):
        return t(v.v)
    src = np.dtype(type(v))
    if t is F32:
        return F32(v)
    if src.kind == "f":
        x = float(v)
        if x != x:
            return t(0)
        lo, hi = (-2 ** 31, 2 ** 31 - 1) if t is I32 else (0, 2 ** 32 - 1)
        x = int(x) if abs(x) < 2 ** 63 else (hi if x > 0 else lo)
        return t(min(max(x, lo), hi))
    return np.asarray(v).astype(np.int64).astype(np.uint32).view(t) if t is I32 else U32(int(v) & 0xFFFFFFFF)


# ---------------------------------------------------------------------------------------
# Interpreter
# ---------------------------------------------------------------------------------------
class Break(Exception):
    pass


class Continue(Exception):
    pass


class Return(Exception):
    def __init__(self, v):
        self.v = v


class Race(RuntimeError):
    pass


class Buffer:
    """A storage buffer: a list of element values (struct dicts or numpy vectors/scalars)."""

    def __init__(self, elems):
        self.e = elems


class Ref:
    """An l-value: buffer element path or local variable path."""

    def __init__(self, kind, root, path):
        self.kind, self.root, self.path = kind, root, path


class Module:
    def __init__(self, src):
        self.decls = Parser(src).module()
        self.structs, self.fns, self.consts, self.globals = {}, {}, {}, {}
        for d in self.decls:
            if d[0] == "struct":
                self.structs[d[1]] = d[2]
            elif d[0] == "fn":
                self.fns[d[1]] = d
            elif d[0] == "const":
                self.consts[d[1]] = d
            elif d[0] == "var":
                self.globals[d[1]] = d

    # -- zero values of types --
    def zero(self, ty):
        name, args = ty
        if name in SCALAR:
            return SCALAR[name](0)
        if name == "bool":
            return False
        if name in ("vec2", "vec3", "vec4"):
            return np.zeros(int(name[3]), dtype=SCALAR[args[0][0]])
        if name == "mat4x4":
            return np.zeros((4, 4), dtype=F32)
        if name in self.structs:
            return {f: self.zero(t) for f, t in self.structs[name]}
        raise TypeError(f"no zero value for {ty}")


class Invocation:
    """One shader invocation's execution state over shared memory with a write overlay."""

    def __init__(self, mod: Module, mem, gid):
        self.m, self.mem, self.gid = mod, mem, gid
        self.overlay = {}  # (buffer name, index) -> element (this invocation's writes)
        self.private = {}

    # -- memory --
    def load_elem(self, buf, idx):
        key = (buf, idx)
        if key in self.overlay:
            return self.overlay[key]
        return self.mem.buffers[buf].e[idx]

    def elem_for_write(self, buf, idx):
        key = (buf, idx)
        if key not in self.overlay:
            self.overlay[key] = copy.deepcopy(self.mem.buffers[buf].e[idx])
        return self.overlay[key]

    # -- evaluation --
    def lookup(self, scopes, name):
        for s in reversed(scopes):
            if name in s:
                return s[name]
        if name in self.m.consts:
            _, _, ty, init = self.m.consts[name]
            v = self.eval(init, [{}])
            return convert(SCALAR[ty[0]], v) if ty and ty[0] in SCALAR else v
        if name in self.mem.uniforms:
            return self.mem.uniforms[name]
        if name in self.m.globals:
            d = self.m.globals[name]
            if d[2] and d[2][0] == "private":
                if name not in self.private:
                    self.private[name] = self.eval(d[4], [{}]) if d[4] else self.m.zero(d[3])
                return self.private[name]
        raise NameError(name)

    def eval(self, e, scopes):
        k = e[0]
        if k == "lit":
            return lit(e[1])
        if k == "bool":
            return e[1]
        if k == "id":
            if e[1] in self.mem.buffers:
                return ("bufref", e[1])
            return self.lookup(scopes, e[1])
        if k == "bin":
            if e[1] in ("&&", "||"):
                a = self.eval(e[2], scopes)
                if e[1] == "&&" and not a:
                    return False
                if e[1] == "||" and a:
                    return True
                return bool(self.eval(e[3], scopes))
            return binop(e[1], self.eval(e[2], scopes), self.eval(e[3], scopes))
        if k == "un":
            v = self.eval(e[2], scopes)
            if e[1] == "-":
                if isinstance(v, Abstract):
                    return Abstract(-v.v)
                return binop("-", type(v)(0) if not is_vec(v) else np.zeros_like(v), v) if np.dtype(
                    v.dtype if is_vec(v) else type(v)).kind != "f" else (-v).astype(F32) if is_vec(v) else F32(-v)
            if e[1] == "!":
                return not v
            if e[1] == "&":
                return v
            raise NotImplementedError(e[1])
        if k == "member":
            base = self.eval(e[1], scopes)
            return self.member(base, e[2])
        if k == "index":
            base = self.eval(e[1], scopes)
            idx = int(default_concrete(self.eval(e[2], scopes)))
            if isinstance(base, tuple) and base[0] == "bufref":
                return copy.deepcopy(self.load_elem(base[1], idx))
            v = base[idx]
            return v.copy() if is_vec(v) else v
        if k == "call":
            return self.call(e[1], e[2], [self.eval(a, scopes) for a in e[3]], e[3], scopes)
        raise NotImplementedError(k)

    @staticmethod
    def member(base, name):
        if isinstance(base, dict):
            v = base[name]
            return v.copy() if is_vec(v) else v
        idx = "xyzw".index(name) if len(name) == 1 else None
        if idx is not None:
            return base[idx]
        return np.array([base["xyzw".index(c)] for c in name], dtype=base.dtype)  # swizzle

    def call(self, name, targs, args, arg_exprs, scopes):
        if name in ("vec2", "vec3", "vec4"):
            n = int(name[3])
            comps = []
            for a in args:
                comps.extend(list(a) if is_vec(a) else [a])
            if len(comps) == 1:
                comps = comps * n
            if targs:
                t = SCALAR[targs[0][0]]
            else:
                concrete = [c for c in comps if not isinstance(c, Abstract)]
                t = type(concrete[0]) if concrete else None
                if t is None:  # all abstract: stays abstract until concretized (float -> f32)
                    t = F32 if any(isinstance(c.v, float) for c in comps) else I32
            return np.array([c.v if isinstance(c, Abstract) else c for c in comps], dtype=t)
        if name == "array":
            return [a for a in args]
        if name in SCALAR:
            return convert(SCALAR[name], args[0])
        if name == "arrayLength":
            return U32(len(self.mem.buffers[args[0][1]].e))
        if name == "abs":
            v = args[0]
            return np.abs(v).astype(v.dtype) if is_vec(v) else type(v)(abs(v))
        if name == "sqrt":
            return F32(np.sqrt(F32(default_concrete(args[0]))))
        if name == "dot":
            a, b = args
            acc = binop("*", a[0], b[0])
            for i in range(1, len(a)):
                acc = binop("+", acc, binop("*", a[i], b[i]))
            return acc
        if name == "clamp":
            x, lo, hi = args
            lo, hi = concretize(lo, x), concretize(hi, x)
            if x < lo:
                return lo
            if x > hi:
                return hi
            return x
        if name in ("min", "max"):
            a, b = args
            a, b = concretize(a, b), concretize(b, a)
            if a != a:
                return b
            if b != b:
                return a
            return (a if a < b else b) if name == "min" else (a if a > b else b)
        if name == "mix":
            a, b, t = args
            t = default_concrete(t)
            a = np.array([x.v if isinstance(x, Abstract) else x for x in a], dtype=F32) if not is_vec(a) else a.astype(F32)
            b = np.array([x.v if isinstance(x, Abstract) else x for x in b], dtype=F32) if not is_vec(b) else b.astype(F32)
            one_minus = F32(F32(1.0) - t)
            return (a * one_minus + b * t).astype(F32)
        if name in self.m.fns:
            return self.call_fn(name, args)
        raise NotImplementedError(f"builtin {name}")

    def call_fn(self, name, args, gen=False):
        _, _, params, ret, body, _ = self.m.fns[name]
        scope = {}
        for (pname, pty), a in zip(params, args):
            scope[pname] = default_concrete(a) if not (pty[0] in SCALAR) else convert(SCALAR[pty[0]], a) \
                if isinstance(a, Abstract) else a
        try:
            self.exec_block(body[1], [scope])
        except Return as r:
            return r.v
        return None

    # -- l-values --
    def ref(self, e, scopes):
        path = []
        while e[0] in ("member", "index"):
            if e[0] == "member":
                path.append(("m", e[2]))
            else:
                path.append(("i", int(default_concrete(self.eval(e[2], scopes)))))
            e = e[1]
        path.reverse()
        assert e[0] == "id", e
        name = e[1]
        if name in self.mem.buffers:
            assert path and path[0][0] == "i"
            return Ref("buf", (name, path[0][1]), path[1:])
        for s in reversed(scopes):
            if name in s:
                return Ref("local", (s, name), path)
        raise NameError(name)

    def store(self, r: Ref, value):
        if r.kind == "buf":
            buf, idx = r.root
            if not r.path:
                key = (buf, idx)
                self.overlay[key] = copy.deepcopy(value)
                return
            cont = self.elem_for_write(buf, idx)
            path = r.path
        else:
            s, name = r.root
            if not r.path:
                old = s[name]
                s[name] = self.cast_like(value, old)
                return
            cont = s[name]
            path = r.path
        for kind, key in path[:-1]:
            cont = cont[key] if kind == "i" else (cont[key] if isinstance(cont, dict) else cont["xyzw".index(key)])
        kind, key = path[-1]
        if kind == "m" and not isinstance(cont, dict):
            key = "xyzw".index(key)
        old = cont[key]
        cont[key] = self.cast_like(value, old)

    @staticmethod
    def cast_like(value, old):
        if isinstance(value, Abstract):
            if is_vec(old):
                return np.full_like(old, value.v)
            return type(old)(value.v)
        if is_vec(old) and is_vec(value):
            return value.astype(old.dtype)
        return value

    def load_ref(self, r: Ref):
        if r.kind == "buf":
            v = self.load_elem(*r.root)
        else:
            s, name = r.root
            v = s[name]
        for kind, key in r.path:
            if kind == "m" and not isinstance(v, dict):
                key = "xyzw".index(key)
            v = v[key]
        return v.copy() if is_vec(v) else copy.deepcopy(v) if isinstance(v, dict) else v

    # -- statements --
    def exec_block(self, stmts, scopes):
        scopes = scopes + [{}]
        for st in stmts:
            self.exec(st, scopes)

    def exec(self, st, scopes):
        k = st[0]
        if k == "decl":
            _, kw, name, ty, init = st
            if init is None:
                v = self.m.zero(ty)
            else:
                v = self.eval(init, scopes)
                if ty is not None and ty[0] in SCALAR:
                    v = convert(SCALAR[ty[0]], v) if isinstance(v, Abstract) else v
                else:
                    v = default_concrete(v) if isinstance(v, Abstract) else v
                if isinstance(v, np.ndarray) and kw != "let":
                    v = v.copy()
            scopes[-1][name] = v
        elif k == "assign":
            _, op, lhs, rhs = st
            r = self.ref(lhs, scopes)
            val = self.eval(rhs, scopes)
            if op != "=":
                cur = self.load_ref(r)
                val = binop(op[0], cur, val)
            self.store(r, val)
        elif k == "expr":
            self.eval(st[1], scopes)
        elif k == "if":
            if self.eval(st[1], scopes):
                self.exec(st[2], scopes)
            elif st[3] is not None:
                self.exec(st[3], scopes)
        elif k == "block":
            self.exec_block(st[1], scopes)
        elif k == "for":
            _, init, cond, upd, body = st
            scopes = scopes + [{}]
            if init:
                self.exec(init, scopes)
            while cond is None or self.eval(cond, scopes):
                try:
                    self.exec_block(body[1], scopes)
                except Break:
                    break
                except Continue:
                    pass
                if upd:
                    self.exec(upd, scopes)
        elif k == "break":
            raise Break()
        elif k == "continue":
            raise Continue()
        elif k == "return":
            raise Return(None if st[1] is None else self.eval(st[1], scopes))
        else:
            raise NotImplementedError(k)

    def entry_steps(self, name):
        """Generator over the entry function's top-level statements (lockstep schedule)."""
        _, _, params, _, body, _ = self.m.fns[name]
        scope = {params[0][0]: np.array([self.gid, 0, 0], dtype=U32)}
        scopes = [scope, {}]
        try:
            for st in body[1]:
                self.exec(st, scopes)
                yield True
        except Return:
            return


class Dispatch:
    """Runs entry points over a grid of invocations on shared buffers (see module docstring)."""

    def __init__(self, mod: Module, buffers: dict, uniforms: dict):
        self.m = mod
        self.buffers = buffers
        self.uniforms = uniforms

    def commit(self, invs):
        seen = {}
        for inv in invs:
            for key, val in inv.overlay.items():
                if key in seen and not equal_values(seen[key], val):
                    raise Race(f"two invocations write {key}")
                seen[key] = val
        for (buf, idx), val in seen.items():
            self.buffers[buf].e[idx] = val
        for inv in invs:
            inv.overlay = {}

    def run(self, entry, invocations, schedule="isolated"):
        invs = [Invocation(self.m, self, gid) for gid in range(invocations)]
        if schedule == "isolated":
            for inv in invs:
                for _ in inv.entry_steps(entry):
                    pass
            self.commit(invs)
        elif schedule == "lockstep":
            gens = [inv.entry_steps(entry) for inv in invs]
            live = list(range(len(invs)))
            while live:
                nxt = []
                for j in live:
                    if next(gens[j], None) is not None:
                        nxt.append(j)
                self.commit([invs[j] for j in live])
                live = nxt
        else:
            raise ValueError(schedule)


def equal_values(a, b):
    if isinstance(a, dict):
        return all(equal_values(a[k], b[k]) for k in a)
    return np.array_equal(np.asarray(a).view(np.uint32) if np.asarray(a).dtype.itemsize == 4 else np.asarray(a),
                          np.asarray(b).view(np.uint32) if np.asarray(b).dtype.itemsize == 4 else np.asarray(b))
