"""Every `Base64.cpp:a-b` citation in the tree points at the lines it claims.

The spans below are the reference file's own (commonLib/cpp_utils/Base64.cpp, 217
lines). A citation must lie inside the file and start and end inside a named span;
when the citing line (or, naming none, the two after it, where a definition follows
a comment) names a codec function, the range must overlap that function's span. When
the reference checkout is present (the build container, never the GPU box) the
spans themselves are checked against it: each span's first line holds its name.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/commonLib/cpp_utils/Base64.cpp"
N_LINES = 217

# name -> (first line, last line, text on the first line)
SPANS = {
    "from_base64": (20, 27, "from_base64[]"),
    "to_base64": (29, 32, "to_base64[]"),
    "numDigits": (37, 46, "Base64::numDigits"),
    "float2int": (48, 78, "Base64::float2int"),
    "int2float": (80, 103, "Base64::int2float"),
    "encode": (104, 169, "Base64::encode"),
    "decode": (171, 217, "Base64::decodeFloat"),
}
# words in the citing text -> the span they name
ALIASES = {
    "numDigits": "numDigits", "num_digits": "numDigits",
    "float2int": "float2int", "int2float": "int2float",
    # the tables are also cited at their use sites in encode / decode
    "from_base64": ("from_base64", "decode"), "to_base64": ("to_base64", "encode"),
    "decodeFloat": "decode", "decodeInt": "decode", "decode_floats": "decode", "decode_ints": "decode",
    "b64_decode": "decode", "encode_floats": "encode", "encode_ints": "encode", "b64_encode": "encode",
}
CITE = re.compile(r"Base64\.cpp:([0-9][-0-9, ]*[0-9]|[0-9])")


def _ranges(spec):
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        a, _, b = part.partition("-")
        yield int(a), int(b or a)


def _tracked_citations():
    out = subprocess.check_output(
        ["git", "grep", "-nE", r"Base64\.cpp:[0-9]", "--", ".", ":!VERDICT.md", ":!SURVEY.md", ":!ADVICE.md",
         ":!BASELINE.md", ":!profiles", ":!*.json", ":!tests/test_citations.py"], cwd=ROOT).decode()
    for line in out.splitlines():
        path, lineno, _ = line.split(":", 2)
        yield path, int(lineno)


def _named(text):
    """Spans the text names: one tuple of acceptable spans per named function."""
    out = set()
    for w in re.findall(r"[A-Za-z_0-9]+", text):
        if w in ALIASES:
            v = ALIASES[w]
            out.add(v if isinstance(v, tuple) else (v,))
    return out


def _in_span(n):
    return any(a <= n <= b for a, b, _ in SPANS.values())


def test_citations_point_inside_named_spans():
    cites = list(_tracked_citations())
    assert len(cites) > 20
    bad = []
    for path, lineno in cites:
        lines = open(os.path.join(ROOT, path), encoding="utf-8").read().splitlines()
        named = _named(lines[lineno - 1]) or _named(" ".join(lines[lineno: lineno + 2]))
        for m in CITE.finditer(lines[lineno - 1]):
            for a, b in _ranges(m.group(1)):
                if a == 0:  # "Base64.cpp:20-27, 0xff": a byte value after a range, not a line
                    continue
                if not (1 <= a <= b <= N_LINES and _in_span(a) and _in_span(b)):
                    bad.append(f"{path}:{lineno}: {a}-{b} outside the file's spans")
                elif named and not any(any(SPANS[n][0] <= b and a <= SPANS[n][1] for n in alt) for alt in named):
                    bad.append(f"{path}:{lineno}: {a}-{b} does not overlap {sorted(named)}")
    assert not bad, "\n".join(bad)


@pytest.mark.skipif(not os.path.exists(REF), reason="reference checkout absent (GPU box)")
def test_spans_match_the_reference_file():
    lines = open(REF, encoding="utf-8", errors="replace").read().splitlines()
    assert len(lines) == N_LINES
    for name, (a, b, head) in SPANS.items():
        assert head in lines[a - 1], (name, a, lines[a - 1])
        if name in ("numDigits", "float2int", "int2float"):
            assert lines[b - 1].strip() == "}", (name, b)
