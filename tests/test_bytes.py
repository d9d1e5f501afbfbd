"""plonky2's binary proof serialization (p2v_pack_proof_bytes).  Parity
unpinned: the reference has no binary reader (README.md:27) and no binary fixture exists
offline.  The C++ reader (csrc/circuit.cpp) is checked against an independent Python writer
(support.proof_bytes) through the JSON path: bytes -> packed words == JSON -> packed words, for
std, lookup, real and P2V_EXT_* circuits, plus the truncation / shape error paths."""
import numpy as np
import pytest

from support import gen_circuit, p2v_module, proof_bytes


@pytest.mark.parametrize("args,ext", [((6, 4, 0, 1, 28, 8), 0), ((6, 0, 1, 2, 28, 8), 0), ((8, 4, 0, 1, 28, 8, 0, 1), 0),
                                      ((6, 3, 0, 1, 28, 8, 0, 2, 6, (3, 1)), 6), ((6, 4, 0, 1, 28, 8, 0, 1, 7, (3, 2)), 7)])
def test_bytes_pack_equals_json_pack(args, ext):
    p2v = p2v_module()
    gc = gen_circuit(*args)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, ext)
    for w, ps, fl in ((1, 1, 0), (2, 3, 0), (1, 5, 2)):
        pr = gc.proof(w, ps, flags=fl)
        ref = vk.pack(pr)
        assert np.array_equal(vk.pack_bytes(proof_bytes(pr)), ref)
        assert np.array_equal(vk.pack_bytes(proof_bytes(pr, pi_prefix=True)), ref)


def test_bytes_error_paths():
    p2v = p2v_module()
    gc = gen_circuit(6, 4, 0, 1, 28, 8)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    b = proof_bytes(gc.proof(1, 1))
    nbytes = 8 * (vk.info.proof_words) + vk.info.num_query_rounds * (4 + vk.info.num_fri_steps)
    assert len(b) == nbytes   # every packed word once, plus one sibling-count byte per Merkle proof

    def code(data):
        with pytest.raises(p2v.P2VError) as e:
            vk.pack_bytes(data)
        return e.value.code
    assert code(b[: len(b) // 2]) == p2v.E_PARSE                  # truncated inside the proof
    assert code(b[:-8]) == p2v.E_SHAPE                            # one public input short
    assert code(b + b"\0" * 8 * 3) == p2v.E_SHAPE                 # trailing words
    i = 3 * 32 * 16 + 8 * 2 * (vk.info.num_openings_this + vk.info.num_openings_next) + 32 * 16 * vk.info.num_fri_steps
    i += 8 * vk.info.oracle_widths[0]                             # first initial-tree sibling count
    assert b[i] == vk.info.lde_bits - vk.info.cap_height
    assert code(b[:i] + bytes([b[i] + 1]) + b[i + 1:]) == p2v.E_SHAPE
    pre = proof_bytes(gc.proof(1, 1), pi_prefix=True)
    bad = bytearray(pre)
    bad[-8 * 5] ^= 1                                              # count 4 -> 5
    assert code(bytes(bad)) == p2v.E_SHAPE
    # values >= p are reduced like the JSON path reduces them
    import struct
    j = len(b) - 8
    (x,) = struct.unpack("<Q", b[j:])
    big = b[:j] + struct.pack("<Q", x + 0xFFFFFFFF00000001) if x < 0xFFFFFFFF else b
    assert np.array_equal(vk.pack_bytes(big), vk.pack_bytes(b))


def test_bytes_fuzz_never_crashes():
    """Seeded truncations and byte flips of a binary proof: the reader returns OK, E_PARSE or
    E_SHAPE, never reads past the buffer (ASan-free host build, so a crash would show here)."""
    import random
    p2v = p2v_module()
    gc = gen_circuit(6, 4, 1, 1, 28, 8)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    b = proof_bytes(gc.proof(1, 1))
    rnd = random.Random(7)
    seen = set()
    for _ in range(300):
        d = bytearray(b)
        op = rnd.randrange(3)
        if op == 0:
            d = d[: rnd.randrange(len(d))]
        elif op == 1:
            for _ in range(rnd.randrange(1, 6)):
                d[rnd.randrange(len(d))] = rnd.randrange(256)
        else:
            i = rnd.randrange(len(d))
            d = d[:i] + bytes(rnd.randrange(1, 40)) + d[i:]
        try:
            vk.pack_bytes(bytes(d))
            seen.add(0)
        except p2v.P2VError as e:
            assert e.code in (p2v.E_PARSE, p2v.E_SHAPE), e
            seen.add(e.code)
    assert {p2v.E_PARSE, p2v.E_SHAPE} <= seen


def test_c_host_bytes_mode_equals_json_mode(tmp_path):
    """examples/p2v_verify.c --bytes (plonky2 binary proofs, p2v_pack_proof_bytes) with --ext 7 (the
    P2V_EXT_* conventions through p2v_circuit_from_json_ex) packs the same words as the JSON mode."""
    import os
    import subprocess
    p2v = p2v_module()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "plonky2-verifier_amd", "p2v_verify")
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "plonky2-verifier_amd"), "p2v_verify"])
    gc = gen_circuit(6, 4, 0, 1, 28, 8, 0, 1, 7, (3, 2))
    (tmp_path / "c.json").write_bytes(gc.common)
    (tmp_path / "v.json").write_bytes(gc.vkey)
    js, bs = [], []
    for i, pr in enumerate([gc.proof(1, 1), gc.proof(2, 2)]):
        (tmp_path / f"p{i}.json").write_bytes(pr)
        (tmp_path / f"p{i}.bin").write_bytes(proof_bytes(pr, pi_prefix=bool(i)))
        js.append(str(tmp_path / f"p{i}.json"))
        bs.append(str(tmp_path / f"p{i}.bin"))
    hdr = [str(tmp_path / "c.json"), str(tmp_path / "v.json")]
    a = subprocess.run([exe, "--ext", "7", "--pack-only", "--dump", str(tmp_path / "a.out")] + hdr + js, capture_output=True, text=True)
    b = subprocess.run([exe, "--bytes", "--ext", "7", "--pack-only", "--dump", str(tmp_path / "b.out")] + hdr + bs,
                       capture_output=True, text=True)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    da, db = np.fromfile(tmp_path / "a.out", np.uint64), np.fromfile(tmp_path / "b.out", np.uint64)
    assert da.size == 2 * p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, 7).info.proof_words
    assert np.array_equal(da, db)
    # without the flags the MinSize circuit is the reference's circuit error (exit 3)
    assert subprocess.run([exe, "--pack-only"] + hdr + js, capture_output=True).returncode == 3
