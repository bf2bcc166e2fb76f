"""Minimal Go expression / composite-literal reader used to extract golden vectors.

Reads the reference's ``*_test.go`` files AS TEXT (study, not execution) and
evaluates the table-driven test literals into plain Python values:

* struct literal  ``pkg.T{A: x}``          → ``{"__type__": "pkg.T", "A": x}``
* slice / array   ``[]T{a, b}``            → ``[a, b]`` (elided element types inherit ``T``)
* map             ``map[K]V{k: v}``        → ``{k: v}`` (insertion order kept)
* ``&x`` / ``*x``                          → ``x`` (pointers are transparent)
* calls                                     → dispatched to Python stand-ins of the
  test helpers / k8s constructors registered by the caller (``funcs``)
* selectors (``corev1.TaintEffectNoSchedule``) → looked up in ``consts``

Only the subset of Go used by the reference's scheduler tests is supported;
anything else raises, so extraction never silently guesses.
"""

from __future__ import annotations

import re

_TOKEN_RE = re.compile(
    r"""
    (?P<ws>\s+)
  | (?P<lcomment>//[^\n]*)
  | (?P<bcomment>/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:[^"\\\n]|\\.)*")
  | (?P<rune>'(?:[^'\\\n]|\\.)')
  | (?P<num>(?:0[xX][0-9a-fA-F_]+)|(?:[0-9][0-9_]*\.[0-9]*(?:[eE][+-]?[0-9]+)?)|(?:\.[0-9]+)|(?:[0-9][0-9_]*(?:[eE][+-]?[0-9]+)?))
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>:=|\.\.\.|&&|\|\||==|!=|<=|>=|<<|>>|\+\+|--|[{}()\[\],:;.&*+\-/%<>=!|^])
    """,
    re.VERBOSE | re.DOTALL,
)


class Tok:
    __slots__ = ("kind", "val", "pos")

    def __init__(self, kind, val, pos):
        self.kind, self.val, self.pos = kind, val, pos

    def __repr__(self):
        return f"{self.kind}:{self.val}"


def tokenize(src: str):
    out = []
    pos = 0
    while pos < len(src):
        m = _TOKEN_RE.match(src, pos)
        if not m:
            raise SyntaxError(f"cannot tokenize at {pos}: {src[pos:pos + 40]!r}")
        kind = m.lastgroup
        val = m.group(kind)
        if kind not in ("ws", "lcomment", "bcomment"):
            out.append(Tok(kind, val, pos))
        pos = m.end()
    out.append(Tok("eof", "", pos))
    return out


def _unquote(s: str) -> str:
    if s.startswith("`"):
        return s[1:-1]
    body = s[1:-1]
    return bytes(body, "utf-8").decode("unicode_escape")


class Parser:
    """Recursive-descent reader producing AST tuples."""

    def __init__(self, toks, i=0):
        self.t = toks
        self.i = i

    def peek(self, k=0):
        return self.t[self.i + k]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, val):
        tok = self.next()
        if tok.val != val:
            raise SyntaxError(f"expected {val!r} got {tok.val!r} at {tok.pos}")
        return tok

    def accept(self, val):
        if self.peek().val == val:
            self.i += 1
            return True
        return False

    # ---- types ---------------------------------------------------------
    def parse_type(self):
        tok = self.peek()
        if tok.val == "[":
            self.next()
            if self.accept("]"):
                return ("slice", self.parse_type())
            n = self.next()
            self.expect("]")
            return ("array", n.val, self.parse_type())
        if tok.val == "map":
            self.next()
            self.expect("[")
            k = self.parse_type()
            self.expect("]")
            return ("map", k, self.parse_type())
        if tok.val == "*":
            self.next()
            return ("ptr", self.parse_type())
        if tok.val == "struct":
            self.next()
            self.expect("{")
            names = []
            while not self.accept("}"):
                group = [self.next().val]
                while self.accept(","):
                    group.append(self.next().val)
                self.parse_type()
                names.extend(group)
                self.accept(";")
            return ("struct", tuple(names))
        if tok.val == "func":
            self.next()
            self._skip_balanced("(", ")")
            # optional result type(s)
            if self.peek().val == "(":
                self._skip_balanced("(", ")")
            elif self.peek().kind == "ident" or self.peek().val in ("[", "*", "map"):
                self.parse_type()
            return ("func",)
        if tok.kind == "ident":
            name = self.next().val
            if self.peek().val == "." and self.peek(1).kind == "ident":
                self.next()
                name = name + "." + self.next().val
            return ("named", name)
        raise SyntaxError(f"bad type at {tok.pos}: {tok.val!r}")

    def _skip_balanced(self, open_, close):
        self.expect(open_)
        depth = 1
        while depth:
            tok = self.next()
            if tok.val == open_:
                depth += 1
            elif tok.val == close:
                depth -= 1
            elif tok.kind == "eof":
                raise SyntaxError("unbalanced")

    # ---- expressions ----------------------------------------------------
    def parse_expr(self):
        left = self.parse_unary()
        while self.peek().val in ("+", "-", "*", "/"):
            op = self.next().val
            right = self.parse_unary()
            left = ("binop", op, left, right)
        return left

    def parse_unary(self):
        tok = self.peek()
        if tok.val == "&":
            self.next()
            return ("addr", self.parse_unary())
        if tok.val == "*":
            self.next()
            return ("deref", self.parse_unary())
        if tok.val == "-":
            self.next()
            return ("neg", self.parse_unary())
        return self.parse_postfix(self.parse_primary())

    def parse_primary(self):
        tok = self.peek()
        if tok.kind in ("str", "raw"):
            self.next()
            return ("lit", _unquote(tok.val))
        if tok.kind == "num":
            self.next()
            v = tok.val.replace("_", "")
            if re.fullmatch(r"0[xX][0-9a-fA-F]+", v):
                return ("lit", int(v, 16))
            if any(ch in v for ch in ".eE") and not v.startswith("0x"):
                return ("lit", float(v))
            return ("lit", int(v))
        if tok.val == "(":
            self.next()
            e = self.parse_expr()
            self.expect(")")
            return e
        if tok.val in ("[", "map", "struct") or (tok.val == "func" and self.peek(1).val == "("):
            if tok.val == "func":
                # func literal: func(...) T { body }  — body kept as opaque tokens
                self.parse_type()
                start = self.i
                self._skip_balanced("{", "}")
                return ("funclit", start)
            typ = self.parse_type()
            if self.peek().val == "{":
                return self.parse_composite(typ)
            return ("type", typ)
        if tok.kind == "ident":
            self.next()
            node = ("ident", tok.val)
            return node
        raise SyntaxError(f"unexpected {tok.val!r} at {tok.pos}")

    def parse_postfix(self, node):
        while True:
            tok = self.peek()
            if tok.val == "." and self.peek(1).kind == "ident":
                self.next()
                name = self.next().val
                if node[0] == "ident":
                    node = ("ident", node[1] + "." + name)
                else:
                    node = ("field", node, name)
            elif tok.val == "(":
                self.next()
                args = []
                while not self.accept(")"):
                    args.append(self.parse_expr())
                    self.accept("...")
                    if not self.accept(","):
                        self.expect(")")
                        break
                node = ("call", node, args)
            elif tok.val == "{" and node[0] == "ident" and self._looks_like_composite():
                node = self.parse_composite(("named", node[1]))
            elif tok.val == "[":
                self.next()
                idx = self.parse_expr()
                self.expect("]")
                node = ("index", node, idx)
            else:
                return node

    def _looks_like_composite(self):
        # Type{...}: the identifier is a type name when followed by '{' in expression context.
        return True

    def parse_composite(self, typ):
        self.expect("{")
        elems = []
        positions = []
        while not self.accept("}"):
            positions.append(self.peek().pos)
            if self.peek().val == "{":
                val = ("elided", self._parse_elided_body())
                key = None
            else:
                first = self.parse_expr_or_elided()
                if self.accept(":"):
                    key = first
                    if self.peek().val == "{":
                        val = ("elided", self._parse_elided_body())
                    else:
                        val = self.parse_expr_or_elided()
                else:
                    key, val = None, first
            elems.append((key, val))
            if not self.accept(","):
                self.expect("}")
                break
        return ("composite", typ, elems, positions)

    def parse_expr_or_elided(self):
        if self.peek().val == "{":
            return ("elided", self._parse_elided_body())
        return self.parse_expr()

    def _parse_elided_body(self):
        node = self.parse_composite(None)
        return node[2]


class Evaluator:
    def __init__(self, consts=None, funcs=None, env=None):
        self.consts = dict(consts or {})
        self.funcs = dict(funcs or {})
        self.env = dict(env or {})

    def eval(self, node, typ=None):
        kind = node[0]
        if kind == "lit":
            return node[1]
        if kind == "ident":
            name = node[1]
            if name in self.env:
                return self.env[name]
            if name in self.consts:
                return self.consts[name]
            if name in ("nil",):
                return None
            if name == "true":
                return True
            if name == "false":
                return False
            raise KeyError(f"unknown identifier {name}")
        if kind in ("addr", "deref"):
            return self.eval(node[1], typ)
        if kind == "neg":
            return -self.eval(node[1])
        if kind == "binop":
            a, b = self.eval(node[2]), self.eval(node[3])
            return {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b,
                    "/": lambda: a // b if isinstance(a, int) else a / b}[node[1]]()
        if kind == "call":
            fn = node[1]
            args = [self.eval(a) for a in node[2]]
            if fn[0] == "ident" and fn[1] in self.funcs:
                return self.funcs[fn[1]](*args)
            if fn[0] == "type":  # conversion like []string(x)
                return args[0]
            raise KeyError(f"unknown function {fn}")
        if kind == "composite":
            return self._composite(node[1], node[2])
        if kind == "elided":
            return self._composite(typ, node[1])
        if kind == "field":
            base = self.eval(node[1])
            return base[node[2]]
        if kind == "index":
            return self.eval(node[1])[self.eval(node[2])]
        raise KeyError(f"cannot evaluate {kind}")

    def _composite(self, typ, elems):
        if typ is None:
            raise SyntaxError("elided composite without known type")
        if typ[0] == "ptr":
            typ = typ[1]
        if typ[0] in ("slice", "array"):
            et = typ[-1]
            return [self.eval(v, et) for _, v in elems]
        if typ[0] == "map":
            kt, vt = typ[1], typ[2]
            out = {}
            for k, v in elems:
                out[self.eval(k, kt)] = self.eval(v, vt)
            return out
        if typ[0] == "named":
            name = typ[1]
            if name in self.consts and isinstance(self.consts[name], tuple):
                # named alias for a container type, e.g. framework.ClusterScoreList
                return self._composite(self.consts[name], elems)
            out = {"__type__": name}
            for k, v in elems:
                if k is None:
                    raise SyntaxError(f"positional struct literal for {name}")
                out[k[1]] = self.eval(v, None)
            return out
        if typ[0] == "struct":
            out = {"__type__": "struct"}
            for idx, (k, v) in enumerate(elems):
                name = typ[1][idx] if k is None else k[1]
                out[name] = self.eval(v, None)
            return out
        raise SyntaxError(f"unsupported composite type {typ}")


def find_func_body(src: str, name: str):
    """Return the token list of the body of ``func name(...)`` (between braces)."""
    m = re.search(r"^func\s+" + re.escape(name) + r"\s*\(", src, re.M)
    if not m:
        raise KeyError(name)
    toks = tokenize(src[m.start():])
    p = Parser(toks)
    p.expect("func")
    p.next()
    p._skip_balanced("(", ")")
    while p.peek().val != "{":
        p.next()
    start = p.i + 1
    p._skip_balanced("{", "}")
    return toks[start:p.i - 1] + [Tok("eof", "", -1)]
