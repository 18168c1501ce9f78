"""Source checks for hand-written HIP that the compiler gets wrong silently.

hipcc in this image (ROCm 7.2) miscompiles ``__builtin_bit_cast(T, v[i])`` and
``__builtin_bit_cast(T, v.y)`` when ``v`` is an ext_vector value: the result is
element 0 (or an unrelated register), with no diagnostic.  Round 5 hit it in
the on-demand lookup's weight load (scripts/alt_level_diff.py found it: every
pixel of every level off).  Element accesses go through a named scalar first
(``const unsigned w1 = v.y; __builtin_bit_cast(h2_t, w1)``) or through a plain
array.  This test keeps the pattern out of the kernels: a bit-cast whose
operand is a subscript or swizzle of a variable declared with a vector type."""
import glob
import os
import re

import pytest

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd", "csrc")
HIP_VECTORS = {"uint2", "uint3", "uint4", "int2", "int4", "float2", "float4", "half2", "ushort2", "ushort4"}


def _vector_types(text):
    return HIP_VECTORS | set(re.findall(r"typedef\s+[\w\s]+?\s+(\w+)\s+__attribute__\(\(ext_vector_type", text))


def _declared_as_vector(text, name, pos, vtypes):
    """The nearest declaration of `name` before `pos`: a vector-typed scalar
    (not an array of vectors, whose elements are whole vectors)."""
    decl = re.compile(r"\b(\w+)\s+(?:\w+\s*(?:\[[^\]]*\])*\s*(?:=[^,;()]*)?\s*,\s*)*%s\s*(\[[^\]]*\])?\s*[=;,)]"
                      % re.escape(name))
    last = None
    for m in decl.finditer(text, 0, pos):
        if m.group(1) not in ("return", "else", "case", "goto"):
            last = m
    return last is not None and last.group(1) in vtypes and last.group(2) is None


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.hpp"))
                                        + glob.glob(os.path.join(CSRC, "ab", "*.inc"))),
                         ids=os.path.basename)
def test_no_bit_cast_of_vector_elements(path):
    text = open(path).read()
    vtypes = _vector_types(text)
    bad = []
    for m in re.finditer(r"__builtin_bit_cast\(\s*[^,]+,\s*(\w+)\s*(\[[^\]]+\]|\.(?:x|y|z|w)\b)\s*\)", text):
        if _declared_as_vector(text, m.group(1), m.start(), vtypes):
            bad.append("%s:%d %s" % (os.path.basename(path), text[:m.start()].count("\n") + 1, m.group(0)))
    assert not bad, "bit-cast of an ext_vector element (miscompiled to element 0): " + "; ".join(bad)
