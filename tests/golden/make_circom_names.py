#!/usr/bin/env python3
"""Extract every signal and component declaration of the reference's own templates
(/root/reference/circuits/nzcptpl.circom, cbortpl.circom, quinSelector.circom) and its two
helper functions (log2.circom, pow.circom) into tests/golden/circom_names.json: per template
its parameters, its top-level `var` definitions, its signals (name, input / output /
intermediate, array dimensions as expressions), and its components (name, dimensions, the
template they are instantiated from and the arguments, as expressions).

This is data extracted from the reference's text (names, shapes, template calls), not its
source: tests/test_circom_names.py evaluates the expressions for nzcp_live's main and checks
that nzcb/circuit.py write_sym() names every declared signal the way circom's .sym would
(main.<component>[i].<signal>[j]). Run here, where /root/reference exists:
  python3 tests/golden/make_circom_names.py"""
import hashlib
import json
import os
import re

REF = "/root/reference/circuits"
FILES = ("nzcptpl.circom", "cbortpl.circom", "quinSelector.circom")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "circom_names.json")


def strip_comments(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def blocks(text: str, kind: str):
    """(name, params, body) of every `template` / `function` in text."""
    for m in re.finditer(rf"\b{kind}\s+(\w+)\s*\(([^)]*)\)\s*\{{", text):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        params = [p.strip() for p in m.group(2).split(",") if p.strip()]
        yield m.group(1), params, text[m.end():i - 1]


def dims(s: str):
    return [d.strip() for d in re.findall(r"\[([^\]]+)\]", s or "")]


def top_level(body: str) -> str:
    """the body's statements at brace depth 0 (declarations; loops' bodies blanked)"""
    out, depth = [], 0
    for ch in body:
        if ch == "{":
            depth += 1
        if depth == 0:
            out.append(ch)
        if ch == "}":
            depth -= 1
    return "".join(out)


def template_record(params, body):
    top = top_level(body)
    rec = {"params": params, "vars": [], "signals": [], "components": []}
    for m in re.finditer(r"\bvar\s+(\w+)(?:\s*\[[^\]]+\])*\s*=\s*([^;]+);", top):
        rec["vars"].append([m.group(1), m.group(2).strip()])
    for m in re.finditer(r"\bsignal\s+(?:(input|output)\s+)?(\w+)((?:\s*\[[^\]]+\])*)\s*;", body):
        rec["signals"].append([m.group(2), m.group(1) or "intermediate", dims(m.group(3))])
    calls = {}
    for m in re.finditer(r"\b(\w+)((?:\s*\[[^\]]+\])*)\s*=\s*([A-Z]\w*)\s*\(([^;]*)\)\s*;", body):
        calls.setdefault(m.group(1), (m.group(3), m.group(4).strip()))
    for m in re.finditer(r"\bcomponent\s+(\w+)((?:\s*\[[^\]]+\])*)\s*(?:=\s*([A-Z]\w*)\s*\(([^;]*)\))?\s*;", body):
        name = m.group(1)
        tmpl, args = (m.group(3), m.group(4).strip()) if m.group(3) else calls.get(name, (None, ""))
        rec["components"].append([name, dims(m.group(2)), tmpl, args])
    return rec


def main():
    out = {"templates": {}, "sources": {}}
    for f in FILES:
        path = os.path.join(REF, f)
        text = open(path).read()
        out["sources"][f] = hashlib.sha256(text.encode()).hexdigest()
        for name, params, body in blocks(strip_comments(text), "template"):
            out["templates"][name] = template_record(params, body)
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
        fh.write("\n")
    print(f"{len(out['templates'])} templates -> {OUT}")


if __name__ == "__main__":
    main()
