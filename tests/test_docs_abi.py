"""The boundary's documentation cannot drift from the header.

INTEGRATION.md's Rust `extern "C"` block is what a maintainer pastes into the
reference's worker/ and parameter_server/ crates (the surface it binds:
worker_ring.rs:39-94, storage/store.rs:8-35, synchronization/synchronizer.rs:7-21).
Every binding there must exist in include/ono_reduce.h with the same number of
parameters, every buffer size its comments quote must be the header's macro,
and every entry-point count the docs quote must be the header's.  CPU only."""
import os
import re

import ono_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ono_reduce.h")


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _split_top(args: str) -> list[str]:
    """Split a parameter list at top-level commas (nested (), <>, [] kept)."""
    out, depth, cur = [], 0, ""
    for ch in args.replace("->", "  "):  # a Rust return arrow is not a closing bracket
        if ch in "(<[":
            depth += 1
        elif ch in ")>]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out if a.strip()]


def _balanced(text: str, start: int) -> tuple[str, int]:
    """text[start] == '(' -> (contents, index after the closing paren)."""
    depth = 0
    for i in range(start, len(text)):
        if text[i] == "(":
            depth += 1
        elif text[i] == ")":
            depth -= 1
            if depth == 0:
                return text[start + 1:i], i + 1
    raise AssertionError("unbalanced parentheses")


def header_decls() -> dict[str, int]:
    text = re.sub(r"/\*.*?\*/", "", _read("include", "ono_reduce.h"), flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(ono_[a-z0-9_]+)\s*\(", text):
        args, _ = _balanced(text, m.end() - 1)
        params = _split_top(args)
        decls[m.group(1)] = 0 if params == ["void"] else len(params)
    return decls


def header_macros() -> dict[str, int]:
    return {k: int(v) for k, v in re.findall(r"#define\s+(ONO_[A-Z0-9_]+)\s+(\d+)", _read("include", "ono_reduce.h"))}


def rust_bindings() -> list[tuple[str, int, str]]:
    """(name, arity, comment text of the binding's lines) for every `pub fn` of
    INTEGRATION.md's extern "C" block."""
    md = _read("INTEGRATION.md")
    block = md[md.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    out = []
    for m in re.finditer(r"pub fn (ono_[a-z0-9_]+)\s*\(", block):
        args, end = _balanced(block, m.end() - 1)
        semi = block.index(";", end)
        eol = block.find("\n", semi)
        # the binding's own lines (from `pub fn` to the end of the line holding its `;`): trailing comments
        comments = " ".join(re.findall(r"//([^\n]*)", block[m.start():eol if eol >= 0 else len(block)]))
        args = re.sub(r"//[^\n]*", "", args)
        out.append((m.group(1), len(_split_top(args)), comments))
    return out


def test_header_parser_sees_every_exported_function():
    assert sorted(header_decls()) == ono_amd.header_functions()


def test_every_rust_binding_exists_with_the_same_arity():
    decls = header_decls()
    binds = rust_bindings()
    assert len(binds) >= 30
    bad = [(n, a, decls.get(n)) for n, a, _ in binds if decls.get(n) != a]
    assert bad == [], f"INTEGRATION.md bindings that do not match include/ono_reduce.h: {bad}"


def test_buffer_sizes_quoted_in_the_bindings_are_the_header_macros():
    macros = header_macros()
    checked = 0
    for name, _, comment in rust_bindings():
        nums = [int(x) for x in re.findall(r"(\d+)\s*bytes|x\s*(\d+)", comment) for x in x if x]
        if not nums:
            continue
        want = macros["ONO_XGMI_HANDLE_BYTES"] if "xgmi" in name else macros["ONO_UID_BYTES"] if "unique_id" in name else None
        if want is None:
            continue
        assert all(v == want for v in nums), f"{name}: comment quotes {nums}, header says {want}"
        checked += 1
    assert checked >= 3  # unique_id, xgmi_handle, xgmi_connect
    # the prose snippets that size a handle buffer
    md = _read("INTEGRATION.md")
    for m in re.finditer(r"\[0u8;\s*(\d+)\]\s*;\s*//\s*(ONO_[A-Z_]+)", md):
        assert int(m.group(1)) == macros[m.group(2)], m.group(0)
    for m in re.finditer(r"n \* (\d+) bytes", md):
        assert int(m.group(1)) == macros["ONO_XGMI_HANDLE_BYTES"], m.group(0)
    # nothing may still call the xGMI handle a 64-byte blob (64 B is the IPC handle inside it)
    for doc in ("INTEGRATION.md", "DESIGN.md", "README.md"):
        text = _read(doc)
        assert not re.search(r"xgmi[^\n]{0,80}\b64[- ]byte handle|handle[^\n]{0,20}\(64 bytes\)|nranks x 64\b", text,
                             re.I), doc


def test_entry_point_counts_quoted_in_the_docs_are_the_headers():
    n = len(header_decls())
    pats = {"INTEGRATION.md": r"emits all (\d+) entry points", "README.md": r"C ABI \((\d+) entry points\)",
            "DESIGN.md": r"C ABI, (\d+) entry points"}
    for doc, pat in pats.items():
        found = re.findall(pat, _read(doc))
        assert found, f"{doc}: no entry-point count found ({pat})"
        assert all(int(x) == n for x in found), f"{doc} quotes {found}, the header declares {n}"


def test_xgmi_timeout_default_quoted_in_the_docs_is_the_librarys():
    src = _read("oxidized-neural-orchestra_amd", "csrc", "ono_xgmi.cpp")
    dflt = float(re.search(r"kDefaultTimeoutS\s*=\s*([\d.]+)", src).group(1))
    for doc in ("DESIGN.md", "INTEGRATION.md", "include/ono_reduce.h"):
        for m in re.finditer(r"(?:TIMEOUT_S|timeout)[^\n]{0,60}?default\s*\(?\s*(\d+)\s*s\b", _read(doc), re.I):
            assert float(m.group(1)) == dflt, f"{doc}: '{m.group(0)}' vs the library's {dflt} s"
