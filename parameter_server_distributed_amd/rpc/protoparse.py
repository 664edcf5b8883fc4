"""A small proto3 parser: ``.proto`` text -> ``FileDescriptorProto`` (no protoc in this image).

Covers the grammar the control plane uses: ``syntax``, ``package``, top-level
``enum`` / ``message`` (scalar, enum and message fields, ``repeated``), unary ``service`` methods,
``//`` and ``/* */`` comments. ``option`` / ``import`` / ``reserved`` statements are accepted and
ignored. Anything else raises ``ProtoSyntaxError`` with the line number, so a schema edit that this
parser does not understand fails loudly instead of being dropped.
"""
from __future__ import annotations

import re

from google.protobuf import descriptor_pb2

F = descriptor_pb2.FieldDescriptorProto
SCALARS = {"int32": F.TYPE_INT32, "int64": F.TYPE_INT64, "uint32": F.TYPE_UINT32, "uint64": F.TYPE_UINT64,
           "sint32": F.TYPE_SINT32, "sint64": F.TYPE_SINT64, "bool": F.TYPE_BOOL, "string": F.TYPE_STRING,
           "bytes": F.TYPE_BYTES, "float": F.TYPE_FLOAT, "double": F.TYPE_DOUBLE, "fixed32": F.TYPE_FIXED32,
           "fixed64": F.TYPE_FIXED64, "sfixed32": F.TYPE_SFIXED32, "sfixed64": F.TYPE_SFIXED64}
_TOKEN = re.compile(r'\s*(?:(//[^\n]*)|(/\*.*?\*/)|("[^"]*")|([A-Za-z_][A-Za-z0-9_.]*)|(-?\d+)|([{}()=;<>,\[\]]))',
                    re.S)


class ProtoSyntaxError(ValueError):
    pass


def _tokens(text: str):
    pos, line = 0, 1
    out = []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            if text[pos:].strip() == "":
                break
            raise ProtoSyntaxError(f"line {line}: unexpected character {text[pos]!r}")
        tok = next(g for g in m.groups() if g is not None) if any(m.groups()) else None
        line += text.count("\n", pos, m.end())
        pos = m.end()
        if tok is None or tok.startswith("//") or tok.startswith("/*"):
            continue
        out.append((tok, line))
    return out


class _P:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self):
        return self.t[self.i][0] if self.i < len(self.t) else None

    def line(self):
        return self.t[min(self.i, len(self.t) - 1)][1] if self.t else 0

    def take(self, want=None):
        if self.i >= len(self.t):
            raise ProtoSyntaxError(f"unexpected end of file (wanted {want!r})")
        tok, ln = self.t[self.i]
        if want is not None and tok != want:
            raise ProtoSyntaxError(f"line {ln}: expected {want!r}, got {tok!r}")
        self.i += 1
        return tok

    def skip_statement(self):
        depth = 0
        while True:
            tok = self.take()
            if tok == "{":
                depth += 1
            elif tok == "}":
                depth -= 1
                if depth <= 0:
                    return
            elif tok == ";" and depth == 0:
                return


def parse(text: str, file_name: str) -> descriptor_pb2.FileDescriptorProto:
    p = _P(_tokens(text))
    fd = descriptor_pb2.FileDescriptorProto(name=file_name)
    pending = []  # (field, type name) resolved once every enum / message name is known
    while p.peek() is not None:
        kw = p.take()
        if kw == "syntax":
            p.take("=")
            s = p.take().strip('"')
            if s != "proto3":
                raise ProtoSyntaxError(f"only proto3 is supported, got {s}")
            fd.syntax = s
            p.take(";")
        elif kw == "package":
            fd.package = p.take()
            p.take(";")
        elif kw in ("option", "import"):
            p.skip_statement()
        elif kw == "enum":
            e = fd.enum_type.add(name=p.take())
            p.take("{")
            while p.peek() != "}":
                if p.peek() in ("option", "reserved"):
                    p.skip_statement()
                    continue
                vn = p.take()
                p.take("=")
                e.value.add(name=vn, number=int(p.take()))
                p.take(";")
            p.take("}")
        elif kw == "message":
            m = fd.message_type.add(name=p.take())
            p.take("{")
            while p.peek() != "}":
                if p.peek() in ("option", "reserved"):
                    p.skip_statement()
                    continue
                label = F.LABEL_OPTIONAL
                if p.peek() == "repeated":
                    p.take()
                    label = F.LABEL_REPEATED
                ftype, ln = p.take(), p.line()
                fname = p.take()
                p.take("=")
                f = m.field.add(name=fname, number=int(p.take()), label=label)
                if p.peek() == "[":  # field options, e.g. [packed = true]
                    while p.take() != "]":
                        pass
                p.take(";")
                if ftype in SCALARS:
                    f.type = SCALARS[ftype]
                else:
                    pending.append((f, ftype, ln))
            p.take("}")
        elif kw == "service":
            s = fd.service.add(name=p.take())
            p.take("{")
            while p.peek() != "}":
                if p.peek() == "option":
                    p.skip_statement()
                    continue
                p.take("rpc")
                meth = s.method.add(name=p.take())
                p.take("(")
                req = p.take()
                p.take(")")
                p.take("returns")
                p.take("(")
                resp = p.take()
                p.take(")")
                if p.peek() == "{":
                    p.skip_statement()
                else:
                    p.take(";")
                meth.input_type, meth.output_type = f".{fd.package}.{req}", f".{fd.package}.{resp}"
            p.take("}")
        else:
            raise ProtoSyntaxError(f"line {p.line()}: unsupported statement {kw!r}")
    enums = {e.name for e in fd.enum_type}
    msgs = {m.name for m in fd.message_type}
    for f, tname, ln in pending:
        base = tname.split(".")[-1]
        if base in enums:
            f.type = F.TYPE_ENUM
        elif base in msgs:
            f.type = F.TYPE_MESSAGE
        else:
            raise ProtoSyntaxError(f"line {ln}: unknown type {tname!r}")
        f.type_name = f".{fd.package}.{base}"
    for s in fd.service:
        for meth in s.method:
            for t in (meth.input_type, meth.output_type):
                if t.split(".")[-1] not in msgs:
                    raise ProtoSyntaxError(f"service {s.name}.{meth.name}: unknown message {t}")
    return fd


def parse_file(path: str) -> descriptor_pb2.FileDescriptorProto:
    import os

    with open(path) as f:
        return parse(f.read(), os.path.basename(path))


def describe(fd: descriptor_pb2.FileDescriptorProto) -> dict:
    """Flat comparable view: {'Msg.field': (number, type, label, type_name)}, enums, methods."""
    out = {}
    for m in fd.message_type:
        out[f"message {m.name}"] = True
        for f in m.field:
            out[f"{m.name}.{f.name}"] = (f.number, f.type, f.label, f.type_name.split(".")[-1])
    for e in fd.enum_type:
        for v in e.value:
            out[f"enum {e.name}.{v.name}"] = v.number
    for s in fd.service:
        for meth in s.method:
            out[f"rpc {s.name}.{meth.name}"] = (meth.input_type.split(".")[-1], meth.output_type.split(".")[-1])
    return out
