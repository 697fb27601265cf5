"""Resolve compile-time A/B switches in a source file (a minimal unifdef):
  python tools/unifdef.py FILE NAME=VALUE ...   (in place)
#if/#elif expressions made only of the given names (and integer literals,
!, &&, ||, ==, !=, <, >, <=, >=, parentheses) are evaluated and the dead arms
dropped; `#ifndef NAME / #define NAME v / #endif` default blocks of a given
name are removed; every occurrence of a given name in code is replaced by its
value.  Other conditionals are kept as they are."""
import re
import sys

path = sys.argv[1]
vals = {}
for a in sys.argv[2:]:
    k, v = a.split("=", 1)
    vals[k] = v
src = open(path).read().split("\n")
NAME = re.compile(r"\b[A-Za-z_]\w*\b")


def evaluate(expr):
    expr = re.sub(r"//.*", "", expr).strip()
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in vals else "__UNKNOWN__", expr)
    names = set(NAME.findall(e))
    if any(n not in vals for n in names):
        return None
    e = NAME.sub(lambda m: "(" + vals[m.group(0)] + ")", e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    return bool(eval(e))


out = []
stack = []   # entries: [mode, taken_any, emitting_parent]; mode: 'keep' (unknown, emit directive) or 'res'


def emitting():
    return all(s["emit"] for s in stack)


i = 0
while i < len(src):
    line = src[i]
    s = line.strip()
    m = re.match(r"#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", s)
    if not m:
        if emitting():
            out.append(NAME.sub(lambda mm: vals.get(mm.group(0), mm.group(0)), line) if vals else line)
        i += 1
        continue
    d, rest = m.group(1), m.group(2).strip()
    if d == "ifndef" and rest.split()[0] in vals if rest else False:
        # default block: #ifndef X / #define X v / #endif  -> drop entirely
        name = rest.split()[0]
        j = i + 1
        while not src[j].strip().startswith("#endif"):
            j += 1
        i = j + 1
        continue
    if d in ("if", "ifdef", "ifndef"):
        if d == "ifdef":
            r = (rest.split()[0] in vals) if rest.split()[0] in vals else None
            r = True if rest.split()[0] in vals else None
        elif d == "ifndef":
            r = None
        else:
            r = evaluate(rest)
        if r is None:
            stack.append(dict(mode="keep", emit=True, taken=False))
            if emitting():
                out.append(line)
        else:
            stack.append(dict(mode="res", emit=r, taken=r))
    elif d == "elif":
        top = stack[-1]
        if top["mode"] == "keep":
            if all(x["emit"] for x in stack[:-1]):
                out.append(line)
        else:
            r = evaluate(rest)
            if r is None:
                raise SystemExit(f"{path}:{i + 1}: unresolvable #elif after a resolved #if")
            top["emit"] = (not top["taken"]) and r
            top["taken"] = top["taken"] or r
    elif d == "else":
        top = stack[-1]
        if top["mode"] == "keep":
            if all(x["emit"] for x in stack[:-1]):
                out.append(line)
        else:
            top["emit"] = not top["taken"]
            top["taken"] = True
    elif d == "endif":
        top = stack.pop()
        if top["mode"] == "keep" and emitting():
            out.append(line)
    i += 1
open(path, "w").write("\n".join(out))
