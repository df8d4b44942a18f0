"""Writes tests/golden/reference_signatures.json: the argument names and defaults of the reference's pybind11 bindings on the
hot path (run in the build container, where /root/reference exists; the tests read only the JSON).

Each `<obj>.def("name", <callable>, "arg"_a [= default], ...)` / `.def(py::init<...>(), ...)` call in the listed binding
files is parsed into {"module", "name", "args": [[name, default-or-null], ...]}; overloads keep their registration
order. Defaults are kept as C++ source text (e.g. "false", "0.f", "open3d::core::Tensor::Eye(4, ...)"); the test maps
them onto Python values. A binding whose arguments are not `_a` literals (positional only) records "args": null.
"""
import json
import os
import re

REF = "/root/reference/cpp/pybind"
HERE = os.path.dirname(os.path.abspath(__file__))
FILES = {
    "geometry/functional/functional.cpp": "nnrt.geometry.functional",
    "geometry/geometry.cpp": "nnrt.geometry",
    "rendering/rendering.cpp": "nnrt.rendering",
    "rendering/functional/functional.cpp": "nnrt.rendering.functional",
    "core/linalg/linalg.cpp": "nnrt.core.linalg",
    "core/core.cpp": "nnrt.core",
}


def _calls(text):
    """Yield (receiver, body) for every `<receiver>.def(` call, body = the text between its parentheses."""
    for m in re.finditer(r"(\w+)\s*\.\s*def\s*\(", text):
        i, depth = m.end(), 1
        in_str = False
        while depth:
            c = text[i]
            if in_str:
                if c == "\\":
                    i += 1
                elif c == '"':
                    in_str = False
            elif c == '"':
                in_str = True
            elif c in "([{<" and c != "<":
                depth += 1
            elif c in ")]}":
                depth -= 1
            i += 1
        yield m.group(1), text[m.end():i - 1]


def _split_top(body):
    """Split on commas at nesting depth 0 (parentheses / braces / template angle brackets of py::overload_cast<...>)."""
    parts, depth, cur, in_str = [], 0, [], False
    for j, c in enumerate(body):
        if in_str:
            cur.append(c)
            if c == '"' and body[j - 1] != "\\":
                in_str = False
            continue
        if c == '"':
            in_str = True
        elif c in "([{<":
            depth += 1
        elif c in ")]}>":
            depth -= 1
        if c == "," and depth == 0:
            parts.append("".join(cur).strip())
            cur = []
        else:
            cur.append(c)
    if cur:
        parts.append("".join(cur).strip())
    return parts


def parse(path, module):
    text = open(path).read()
    text = re.sub(r"//[^\n]*", "", text)
    out = []
    for recv, body in _calls(text):
        parts = _split_top(body)
        if not parts:
            continue
        head = parts[0]
        if head.startswith("py::init"):
            name = "__init__"
        else:
            mm = re.match(r'"([^"]+)"', head)
            if not mm:
                continue
            name = mm.group(1)
        args = []
        for p in parts[1:]:
            am = re.match(r'"(\w+)"_a(?:\s*=\s*(.+))?$', p, re.S)
            if am:
                args.append([am.group(1), None if am.group(2) is None else " ".join(am.group(2).split())])
        positional_only = not args and any(re.match(r'"\w+"$', p) for p in parts[2:])
        out.append(dict(module=module, receiver=recv, name=name, args=None if positional_only else args))
    return out


def main():
    rows = []
    for rel, module in FILES.items():
        rows += parse(os.path.join(REF, rel), module)
    with open(os.path.join(HERE, "reference_signatures.json"), "w") as f:
        json.dump(rows, f, indent=1)
    print(f"{len(rows)} bindings written")


if __name__ == "__main__":
    main()
