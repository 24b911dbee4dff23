"""The Go drop-in (go/) stays buildable under the reference's Go pin.

The reference pins Go 1.11 (go.mod:30 `go 1.11`; CI matrix Go 1.11 and
1.14, .github/workflows/continuous-integration.yml:15; sample/docker/
Dockerfile:2 golang:1.14.4).  There is no Go toolchain in this image, so
this is a source-level check: every .go file under go/ is scanned, with
comments and string literals removed, for APIs and syntax that need a newer
Go, and for the layout rules of the patch (package names of the reference
directories the files go into; the core imports nothing from sample/).
"""
from __future__ import annotations

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go")

# API or syntax -> the Go release that introduced it
POST_111 = [
    (r"\bunsafe\.(Slice|SliceData|String|StringData|Add)\b", "1.17/1.20"),
    (r"\.FillBytes\(", "1.15"),
    (r"\berrors\.(Is|As|Unwrap|Join)\(", "1.13/1.20"),
    (r"\bio\.(ReadAll|Discard|NopCloser)\b", "1.16"),
    (r"\bos\.(ReadFile|WriteFile|ReadDir|DirFS|UserHomeDir|UserConfigDir|UserCacheDir)\b", "1.12-1.16"),
    (r"\b(strings|bytes)\.(ReplaceAll|Cut|CutPrefix|CutSuffix|Clone)\(", "1.12-1.20"),
    (r"\.(Microseconds|Milliseconds)\(\)", "1.13"),
    (r"\btime\.(UnixMilli|UnixMicro)\(", "1.17"),
    (r"\bt\.(Cleanup|TempDir|Setenv)\(", "1.14-1.17"),
    (r"\bb\.(Cleanup|TempDir|Setenv)\(", "1.14-1.17"),
    (r"\bmath\.(MaxInt|MinInt|MaxUint)\b(?!\d)", "1.17"),
    (r"\batomic\.(Int32|Int64|Uint32|Uint64|Bool|Pointer|Value)\{", "1.19"),
    (r"\bsync\.(OnceFunc|OnceValue|OnceValues)\b", "1.21"),
    (r"(?<![\w.])(min|max|clear)\(", "1.21 builtins"),
    (r"\bany\b", "1.18"),
    (r"\bfunc\s+(\(\w+\s+\*?\w+\)\s*)?\w+\[", "1.18 type parameters"),
    (r"\btype\s+\w+\[\w+\s+\w", "1.18 type parameters"),
    (r"\brange\s+\d", "1.22 range over int"),
    (r"\b0[bBoO][0-9a-fA-F]", "1.13 binary / octal literals"),
    (r"\b\d+_\d", "1.13 digit separators"),
    (r"%w", "1.13 error wrapping"),
    (r"^//go:build", "1.17 build constraints"),
]

# the reference directories the files are dropped into, and their package
# names there (api/api.go, core/replica.go, sample/authentication/...,
# sample/peer/cmd/run.go)
PACKAGES = {"api": "api", "core": "minbft", "client": "client", "gpuauth": "gpuauth",
            os.path.join("sample", "peer", "cmd"): "cmd"}


def go_files():
    out = []
    for d, _, fs in os.walk(GO):
        out += [os.path.join(d, f) for f in fs if f.endswith(".go")]
    return sorted(out)


def strip(src: str, keep_strings: bool = False) -> str:
    """Go source without comments and (unless keep_strings) string and rune
    literals."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            # a cgo preamble is C, not Go: drop it too
            i = n if j < 0 else j + 2
        elif c in "\"'`":
            q, j = c, i + 1
            while j < n and src[j] != q:
                j += 2 if (src[j] == "\\" and q != "`") else 1
            out.append(src[i:j + 1] if keep_strings else q + q)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def test_there_are_go_sources():
    names = {os.path.relpath(p, GO) for p in go_files()}
    for want in ("gpuauth/gpuauth.go", "gpuauth/errors.go", "core/message-handling-batch.go",
                 "api/authen-batch.go", "sample/peer/cmd/gpu-stack.go"):
        assert want in names, names


@pytest.mark.parametrize("path", go_files(), ids=lambda p: os.path.relpath(p, GO))
def test_no_post_go111_apis(path):
    raw = open(path).read()
    code = strip(raw)
    with_strings = strip(raw, keep_strings=True)
    bad = []
    for pat, ver in POST_111:
        src = raw if pat.startswith("^//") else with_strings if pat == "%w" else code
        for m in re.finditer(pat, src, flags=re.M):
            line = src[:m.start()].count("\n") + 1
            bad.append(f"{m.group(0)!r} (Go {ver}) near code line {line}")
    assert not bad, bad


@pytest.mark.parametrize("path", go_files(), ids=lambda p: os.path.relpath(p, GO))
def test_shift_counts_are_unsigned_or_constant(path):
    """Go < 1.13 rejects a signed (int) shift count: every shift count is a
    literal, a declared constant, or an explicit uint conversion."""
    code = strip(open(path).read())
    consts = set(re.findall(r"\bconst\s+(\w+)", code))
    for block in re.findall(r"\bconst\s*\((.*?)\)", code, flags=re.S):
        consts |= set(re.findall(r"^\s*(\w+)", block, flags=re.M))
    bad = []
    for m in re.finditer(r"(<<|>>)\s*([A-Za-z_]\w*)", code):
        ident = m.group(2)
        if ident in consts or ident.startswith("uint"):
            continue
        bad.append(m.group(0))
    assert not bad, bad


@pytest.mark.parametrize("path", go_files(), ids=lambda p: os.path.relpath(p, GO))
def test_package_names_and_imports(path):
    rel = os.path.relpath(os.path.dirname(path), GO)
    code = strip(open(path).read())
    pkg = re.search(r"^package\s+(\w+)", code, flags=re.M).group(1)
    assert pkg == PACKAGES[rel], (rel, pkg)
    if rel in ("core", "client"):
        # the core and the client depend on api / messages / usig only, never on a sample
        assert "sample/" not in open(path).read().split("import (", 1)[1].split(")", 1)[0]


def test_go_mod_not_raised():
    """The patch adds no go.mod of its own (it builds inside the reference's
    module, go.mod:30 `go 1.11`)."""
    for d, _, fs in os.walk(GO):
        assert "go.mod" not in fs, d


def test_checker_flags_newer_go():
    """The scan itself catches what round 2's binding used."""
    src = strip('b := unsafe.Slice((*byte)(p), n) // ok in a comment: unsafe.Add\n'
                'sk.D.FillBytes(d)\nx := fmt.Errorf("%w", err)\nvar v any\nn := 1 << k\n')
    hits = {ver for pat, ver in POST_111 if re.search(pat, src, flags=re.M)}
    assert {"1.17/1.20", "1.15", "1.18"} <= hits, hits
    assert re.search(r"(<<|>>)\s*([A-Za-z_]\w*)", src)
    # %w lives in format strings: checked with the literals kept
    assert re.search(r"%w", strip('x := fmt.Errorf("%w", err) // %v', keep_strings=True))
    assert not re.search(r"%w", strip('x := 1 // fmt.Errorf("%w")', keep_strings=True))
