"""Parser for the ACE operator strings pyaceqd writes into param files.

The reference never evaluates these strings itself; it writes them verbatim into `add_Hamiltonian`,
`add_Lindblad`, `add_Pulse`, `add_Output`, `initial`, `apply_Operator` lines
(general_system.py:239-289) and lets ACE parse them. libpqd takes dense matrices, so the strings
are evaluated here. Grammar covered (every form used by the model wrappers: two_level_system/tls.py,
four_level_system/linear.py, six_level_system/linear.py, four_level_system/dark_model.py,
two_time/correlations.py output/MTO strings):

    expr    := kron (('+' | '-') kron)*
    kron    := term ('otimes' term)*
    term    := unary (('*' | '/') unary)*
    unary   := ('-' | '+') unary | atom
    atom    := NUMBER | 'i' | 'pi' | 'hbar' | FUNC '(' expr ')' | '(' expr ')'
             | '|' INT '><' INT '|_' INT | 'Id_' INT | 'n_' INT | 'b_' INT | 'bdagger_' INT
    FUNC    := sqrt | exp | sin | cos

Scalars are complex Python numbers, operators are numpy (d, d) complex arrays; `*` between two
operators is the matrix product, `otimes` the Kronecker product (left factor = most significant).
"""
import cmath
import functools
import re

import numpy as np

from .constants import hbar as HBAR

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<ketbra>\|\s*(?P<k>\d+)\s*><\s*(?P<b>\d+)\s*\|_(?P<kd>\d+))
  | (?P<named>(?:Id|n|bdagger|b)_(?P<nd>\d+))
  | (?P<num>(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)
  | (?P<ident>[A-Za-z_][A-Za-z_0-9]*)
  | (?P<op>[-+*/()])
""", re.VERBOSE)

_FUNCS = {"sqrt": cmath.sqrt, "exp": cmath.exp, "sin": cmath.sin, "cos": cmath.cos}
_CONSTS = {"i": 1j, "pi": np.pi, "hbar": HBAR}


def _tokenize(s):
    pos, out = 0, []
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError(f"cannot parse operator string at {s[pos:]!r} (in {s!r})")
        pos = m.end()
        if m.lastgroup == "ws":
            continue
        if m.group("ketbra"):
            out.append(("ketbra", (int(m.group("k")), int(m.group("b")), int(m.group("kd")))))
        elif m.group("named"):
            name = m.group("named").split("_")[0]
            out.append(("named", (name, int(m.group("nd")))))
        elif m.group("num"):
            out.append(("num", float(m.group("num"))))
        elif m.group("ident"):
            out.append(("ident", m.group("ident")))
        else:
            out.append(("op", m.group("op")))
    out.append(("end", None))
    return out


def _is_op(v):
    return isinstance(v, np.ndarray)


def _basis_op(name, d):
    if name == "Id":
        return np.eye(d, dtype=complex)
    if name == "n":
        return np.diag(np.arange(d, dtype=float)).astype(complex)
    b = np.diag(np.sqrt(np.arange(1, d, dtype=float)), k=1).astype(complex)  # annihilator
    return b if name == "b" else b.conj().T


class _Parser:
    def __init__(self, text):
        self.text = text
        self.toks = _tokenize(text)
        self.i = 0

    def peek(self):
        return self.toks[self.i]

    def take(self, kind=None, val=None):
        t = self.toks[self.i]
        if (kind and t[0] != kind) or (val is not None and t[1] != val):
            raise ValueError(f"unexpected token {t[1]!r} in {self.text!r}")
        self.i += 1
        return t

    def parse(self):
        v = self.expr()
        self.take("end")
        return v

    def expr(self):
        v = self.kron()
        while self.peek() in (("op", "+"), ("op", "-")):
            sign = self.take()[1]
            w = self.kron()
            v = _add(v, w if sign == "+" else _neg(w), self.text)
        return v

    def kron(self):
        v = self.term()
        while self.peek() == ("ident", "otimes"):
            self.take()
            w = self.term()
            if not (_is_op(v) and _is_op(w)):
                raise ValueError(f"'otimes' needs operators on both sides in {self.text!r}")
            v = np.kron(v, w)
        return v

    def term(self):
        v = self.unary()
        while self.peek() in (("op", "*"), ("op", "/")):
            o = self.take()[1]
            w = self.unary()
            if o == "*":
                if _is_op(v) and _is_op(w):
                    if v.shape != w.shape:
                        raise ValueError(f"dimension mismatch {v.shape} * {w.shape} in {self.text!r}")
                    v = v @ w
                else:
                    v = v * w
            else:
                if _is_op(w):
                    raise ValueError(f"division by an operator in {self.text!r}")
                v = v / w
        return v

    def unary(self):
        t = self.peek()
        if t == ("op", "-"):
            self.take()
            return _neg(self.unary())
        if t == ("op", "+"):
            self.take()
            return self.unary()
        return self.atom()

    def atom(self):
        kind, val = self.peek()
        if kind == "num":
            self.take()
            return complex(val)
        if kind == "ketbra":
            self.take()
            k, b, d = val
            if k >= d or b >= d:
                raise ValueError(f"|{k}><{b}|_{d}: index out of range in {self.text!r}")
            m = np.zeros((d, d), dtype=complex)
            m[k, b] = 1.0
            return m
        if kind == "named":
            self.take()
            return _basis_op(*val)
        if kind == "ident":
            self.take()
            if val in _CONSTS:
                return complex(_CONSTS[val])
            if val in _FUNCS:
                self.take("op", "(")
                a = self.expr()
                self.take("op", ")")
                if _is_op(a):
                    raise ValueError(f"{val}() of an operator in {self.text!r}")
                return complex(_FUNCS[val](a))
            raise ValueError(f"unknown identifier {val!r} in {self.text!r}")
        if (kind, val) == ("op", "("):
            self.take()
            v = self.expr()
            self.take("op", ")")
            return v
        raise ValueError(f"unexpected token {val!r} in {self.text!r}")


def _neg(v):
    return -v


def _add(a, b, text):
    if _is_op(a) and _is_op(b):
        if a.shape != b.shape:
            raise ValueError(f"dimension mismatch {a.shape} + {b.shape} in {text!r}")
        return a + b
    if _is_op(a) or _is_op(b):
        raise ValueError(f"adding a scalar to an operator in {text!r}")
    return a + b


def evaluate(text):
    """Evaluate an operator string; returns a complex (d, d) array (or a complex scalar)."""
    return _Parser(str(text)).parse()


def to_matrix(text, dim=None):
    """Operator string -> (dim, dim) complex matrix; a bare scalar is promoted to scalar*Id. Parses are cached per
    (text, dim) (a two-time sweep lowers the same MTO strings once per trajectory); every call returns a fresh array."""
    return _to_matrix_cached(str(text), dim).copy()


@functools.lru_cache(maxsize=4096)
def _to_matrix_cached(text, dim):
    v = evaluate(text)
    if not _is_op(v):
        if dim is None:
            raise ValueError(f"{text!r} is a scalar and no dimension is known")
        return complex(v) * np.eye(dim, dtype=complex)
    if dim is not None and v.shape != (dim, dim):
        raise ValueError(f"{text!r} has dimension {v.shape[0]}, expected {dim}")
    return v


def dimension_of(text):
    v = evaluate(text)
    if not _is_op(v):
        raise ValueError(f"{text!r} is a scalar")
    return v.shape[0]
