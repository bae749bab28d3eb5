#!/usr/bin/env python3
"""Resolve preprocessor conditionals on a fixed set of macros (a small unifdef): the way the rejected
measurement branches of render.hip were stripped (VERDICT r05 "next" 5), their code kept as patches.

    python tools/unifdef.py FILE -D NAME=VALUE ... -U NAME ...   (rewrites FILE in place)

A conditional group (#if / #ifdef / #ifndef ... #elif ... #else ... #endif) is resolved when every
condition in its chain uses only the named macros (plus integer literals, !, &&, ||, ==, !=, <, >,
parentheses, defined()); the kept branch's lines stay, the directives go. Other groups are kept
verbatim (their bodies still processed). Lines `#define NAME` of a named macro are dropped.
"""
from __future__ import annotations

import argparse
import re

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif|define)\b(.*)$")


def evaluate(kind, expr, defs, undefs):
    """True / False, or None when the condition names a macro outside defs / undefs."""
    expr = expr.split("//")[0].strip()
    if kind in ("ifdef", "ifndef"):
        name = expr.split()[0]
        if name in defs:
            val = True
        elif name in undefs:
            val = False
        else:
            return None
        return val if kind == "ifdef" else not val

    def repl_defined(m):
        name = m.group(1) or m.group(2)
        if name in defs:
            return "1"
        if name in undefs:
            return "0"
        raise KeyError(name)

    try:
        e = re.sub(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)", repl_defined, expr)
    except KeyError:
        return None
    for name in re.findall(r"[A-Za-z_]\w*", e):
        if name in defs:
            continue
        if name in undefs:
            continue
        return None
    e = re.sub(r"[A-Za-z_]\w*", lambda m: str(defs.get(m.group(0), 0)), e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    return bool(eval(e, {"__builtins__": {}}))


def process(lines, defs, undefs):
    out = []
    # stack of groups: each {"resolved": bool, "taken": bool (a branch already kept), "active": bool}
    stack = []

    def emitting():
        return all(g["active"] for g in stack)

    for line in lines:
        m = DIRECTIVE.match(line)
        kind = m.group(1) if m else None
        if kind in ("if", "ifdef", "ifndef"):
            v = evaluate(kind, m.group(2), defs, undefs)
            if v is None:
                stack.append({"resolved": False, "taken": True, "active": True})
                if emitting():
                    out.append(line)
            else:
                stack.append({"resolved": True, "taken": v, "active": v})
            continue
        if kind == "elif":
            g = stack[-1]
            if not g["resolved"]:
                if all(x["active"] for x in stack[:-1]):
                    out.append(line)
                continue
            v = evaluate("if", m.group(2), defs, undefs)
            if v is None:
                raise SystemExit(f"unresolvable #elif in a resolved group: {line.strip()}")
            g["active"] = (not g["taken"]) and v
            g["taken"] = g["taken"] or v
            continue
        if kind == "else":
            g = stack[-1]
            if not g["resolved"]:
                if all(x["active"] for x in stack[:-1]):
                    out.append(line)
                continue
            g["active"] = not g["taken"]
            g["taken"] = True
            continue
        if kind == "endif":
            g = stack.pop()
            if not g["resolved"] and emitting():
                out.append(line)
            continue
        if kind == "define":
            name = m.group(2).split()[0] if m.group(2).split() else ""
            if name in defs or name in undefs:
                continue
        if emitting():
            out.append(line)
    if stack:
        raise SystemExit("unbalanced conditionals")
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("file")
    p.add_argument("-D", action="append", default=[])
    p.add_argument("-U", action="append", default=[])
    a = p.parse_args()
    defs = {}
    for d in a.D:
        k, _, v = d.partition("=")
        defs[k] = int(v or "1", 0)
    lines = open(a.file).read().splitlines(keepends=True)
    open(a.file, "w").write("".join(process(lines, defs, set(a.U))))


if __name__ == "__main__":
    main()
