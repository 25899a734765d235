"""The Java drop-ins' constructor defaults equal the reference's (no JDK here, so read the source).

A drop-in that is constructed the way the reference's class is must run what the reference
runs.  The defaults this pins, with the reference lines they restate (under
src/main/java/jwave/transforms/):

* ContinuousWaveletTransform(wavelet) -> PaddingType.SYMMETRIC (ContinuousWaveletTransform.java:91-93);
  (wavelet, paddingType) keeps the caller's padding (:101-106).
* MODWTTransform(wavelet) -> fftConvolutionThreshold 4096 (MODWTTransform.java:144), method AUTO
  (:167); (wavelet, fftThreshold) sets the threshold (:191-194): the second int is the
  threshold, never the arithmetic contract.
* FastWaveletTransform / WaveletPacketTransform / FastFourierTransform (no extra state).
* Every one-argument (or no-argument) drop-in runs JW_ARITH_STRICT, the JVM's arithmetic.

The resolver follows `this(...)` chains by substituting arguments, so a default set two
constructors away is still seen.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JDIR = os.path.join(ROOT, "java", "jwave", "hip")
HEADER = os.path.join(ROOT, "include", "jwave_hip.h")


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
            continue
        depth += ch in "([{"
        depth -= ch in ")]}"
        cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _constructors(cls):
    """[(param names, param types, body)] of every public constructor of java/jwave/hip/<cls>."""
    with open(os.path.join(JDIR, cls + ".java")) as f:
        src = _strip_comments(f.read())
    ctors = []
    for m in re.finditer(r"public\s+%s\s*\(([^)]*)\)\s*\{" % cls, src):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        params = _split_args(m.group(1))
        types = [p.rsplit(None, 1)[0] for p in params]
        names = [p.rsplit(None, 1)[1] for p in params]
        ctors.append((names, types, src[m.end():i - 1]))
    return ctors


def _resolve(cls, types, args):
    """Follow the constructor with these parameter types, called with `args` (Java expressions),
    to the constructor that calls super(...).  Returns (super args, {field: value}), each value
    a Java expression in the caller's terms."""
    ctors = _constructors(cls)
    match = [c for c in ctors if c[1] == types]
    assert len(match) == 1, f"{cls}({', '.join(types)}) not found exactly once"
    names, _, body = match[0]
    env = dict(zip(names, args))

    def subst(expr):
        return re.sub(r"\b\w+\b", lambda w: env.get(w.group(0), w.group(0)), expr).strip()

    t = re.search(r"\bthis\s*\((.*?)\)\s*;", body, flags=re.S)
    if t:
        callee_args = [subst(a) for a in _split_args(t.group(1))]
        # pick the callee by arity (the drop-ins have one constructor per arity)
        cands = [c for c in ctors if len(c[0]) == len(callee_args) and c[0] != names]
        assert len(cands) == 1, f"{cls}: ambiguous this({t.group(1)})"
        return _resolve(cls, cands[0][1], callee_args)
    s = re.search(r"\bsuper\s*\((.*?)\)\s*;", body, flags=re.S)
    sup = [subst(a) for a in _split_args(s.group(1))] if s else []
    fields = {}
    for fm in re.finditer(r"(?:this\.)?(\w+)\s*=\s*([^;=]+);", body):
        fields[fm.group(1)] = subst(fm.group(2))
    # a contract handed straight to the native plan (FWT / WPT) counts as the arith field
    pc = re.search(r"nPlanCreate\((.*?)\)\s*;", body, flags=re.S)
    if pc and "arith" not in fields:
        fields["arith"] = subst(_split_args(pc.group(1))[-1])
    # no constructor may change the reference's own state behind super()
    assert "setConvolutionMethod" not in body and "fftConvolutionThreshold" not in body, cls
    return sup, fields


def _header_define(name):
    with open(HEADER) as f:
        m = re.search(r"#define\s+%s\s+(\d+)" % name, f.read())
    return int(m.group(1))


def test_arith_constants_match_the_c_abi():
    strict = _header_define("JW_ARITH_STRICT")
    for cls in ("HipMODWTTransform", "HipFastWaveletTransform", "HipFastFourierTransform"):
        with open(os.path.join(JDIR, cls + ".java")) as f:
            src = f.read()
        m = re.search(r"ARITH_STRICT\s*=\s*(\d+)", src)
        assert m and int(m.group(1)) == strict, cls


def test_cwt_default_padding_is_symmetric():
    # ContinuousWaveletTransform.java:91-93: this(wavelet, PaddingType.SYMMETRIC)
    sup, fields = _resolve("HipContinuousWaveletTransform", ["ContinuousWavelet"], ["w0"])
    assert sup == ["w0", "PaddingType.SYMMETRIC"]
    assert fields["padding"] == "PaddingType.SYMMETRIC.ordinal()"
    assert fields["arith"] == "HipMODWTTransform.ARITH_STRICT"
    assert fields["device"] == "-1"
    # the ordinal the glue passes is the C-ABI's JW_PAD_SYMMETRIC (enum order ZERO, SYMMETRIC, ...)
    assert _header_define("JW_PAD_SYMMETRIC") == 1 and _header_define("JW_PAD_ZERO") == 0


def test_cwt_two_argument_constructor_keeps_the_callers_padding():
    # ContinuousWaveletTransform.java:101-106
    sup, fields = _resolve("HipContinuousWaveletTransform",
                           ["ContinuousWavelet", "PaddingType"], ["w0", "p0"])
    assert sup == ["w0", "p0"]
    assert fields["padding"] == "p0.ordinal()"
    assert fields["arith"] == "HipMODWTTransform.ARITH_STRICT"


def test_modwt_default_is_reference_threshold_auto_strict():
    # MODWTTransform(wavelet) (:180-183): super(w) keeps fftConvolutionThreshold = 4096 (:144)
    # and ConvolutionMethod.AUTO (:167); the drop-in must not touch either, and runs STRICT.
    sup, fields = _resolve("HipMODWTTransform", ["Wavelet"], ["w0"])
    assert sup == ["w0"]
    assert fields["arith"] == "ARITH_STRICT" and fields["device"] == "-1"


def test_modwt_second_int_is_the_fft_threshold():
    # MODWTTransform(wavelet, fftThreshold) (:191-194): new HipMODWTTransform(w, 8192) must
    # mean threshold 8192, as it does for the reference class.
    sup, fields = _resolve("HipMODWTTransform", ["Wavelet", "int"], ["w0", "8192"])
    assert sup == ["w0", "8192"]
    assert fields["arith"] == "ARITH_STRICT"
    sup, fields = _resolve("HipMODWTTransform", ["Wavelet", "int", "int"], ["w0", "t0", "a0"])
    assert sup == ["w0", "t0"] and fields["arith"] == "a0"


def test_modwt_plan_reads_the_live_threshold_field():
    # the plan takes the protected field (MODWTTransform.java:144), so a subclass or the
    # two-argument constructor's value is what the engine's per-level AUTO rule uses
    with open(os.path.join(JDIR, "HipMODWTTransform.java")) as f:
        src = _strip_comments(f.read())
    assert re.search(r"nPlanCreate\([^;]*fftConvolutionThreshold", src, flags=re.S)
    assert "getConvolutionMethod().ordinal()" in src


@pytest.mark.parametrize("cls,types", [
    ("HipFastWaveletTransform", ["Wavelet"]),
    ("HipWaveletPacketTransform", ["Wavelet"]),
    ("HipFastFourierTransform", []),
])
def test_other_drop_ins_default_to_strict(cls, types):
    args = ["w0"][:len(types)]
    sup, fields = _resolve(cls, types, args)
    assert sup == args
    assert fields["arith"] in ("ARITH_STRICT", "HipFastWaveletTransform.ARITH_STRICT")
    assert fields["device"] == "-1"


def test_every_public_constructor_has_a_reference_counterpart_or_extra_args():
    # a drop-in constructor whose parameter types equal a reference constructor's must mean
    # the same thing; the only extra arities the drop-ins add carry (arith[, device])
    ref = {
        "HipContinuousWaveletTransform": [["ContinuousWavelet"], ["ContinuousWavelet", "PaddingType"]],
        "HipMODWTTransform": [["Wavelet"], ["Wavelet", "int"]],
        "HipFastWaveletTransform": [["Wavelet"]],
        "HipWaveletPacketTransform": [["Wavelet"]],
        "HipFastFourierTransform": [[]],
    }
    for cls, sigs in ref.items():
        have = [c[1] for c in _constructors(cls)]
        for s in sigs:
            assert s in have, f"{cls} lacks the reference constructor ({', '.join(s)})"
        for names, types, _ in _constructors(cls):
            if types in sigs:
                continue
            extra = names[-2:] if names[-1] == "device" else names[-1:]
            assert extra[0] == "arith", f"{cls}({', '.join(types)}) adds {names}"
