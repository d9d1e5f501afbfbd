"""p2v — host-side mirror of the reference verifier's API over libp2v (ctypes).

The reference (bkomuves/plonky2-verifier, Haskell) exposes

    verifyProof :: VerifierCircuitData -> ProofWithPublicInputs -> Bool   (src/Plonk/Verifier.hs:56)

with inputs decoded from JSON by the Types.hs aeson instances (src/Types.hs:47-279).
This module keeps that shape:

    vkey  = VerifierCircuitData.from_json(common_json, vkey_json)      # Types.hs:220-224
    proof = ProofWithPublicInputs.from_json(proof_json)                # Types.hs:245-254
    ok    = verify_proof(vkey, proof)                                  # Plonk/Verifier.hs:56

and adds the batch form the GPU is built for (verify_proof_batch / BatchVerifier).
Where the reference raises `error` (failed Merkle proof, folding-step mismatch, unsupported
circuit) this module raises VerifierError with the same class, and verify_proof returns False
where the reference returns False.  A proof with another number of public inputs or
final-polynomial coefficients than the circuit implies is verified, as the reference verifies
it, against a shape variant of the circuit (p2v_circuit_shape_variant: the packed layout with
those lengths; the reference hashes / evaluates whatever it is given); any other length
mismatch is an `error` in the reference too and raises P2VError(E_SHAPE) at pack time.

All verification runs in libp2v's HIP kernels on MI355X; there is no CPU fallback — on a
machine without a GPU, verification raises P2VError(P2V_E_NODEVICE).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Union

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("P2V_LIB") or os.path.join(_HERE, "libp2v.so")   # P2V_LIB: A/B measurement builds

# per-proof status codes (include/p2v.h)
ACCEPT = 1
REJECT = 0
ERR_INITIAL_MERKLE = -1
ERR_STEP_MERKLE = -2
ERR_STEP_EVAL = -3
ERR_STEP_ARITY = -4
ERR_SHAPE = -5
ERR_CIRCUIT = -6
ERR_PARSE = -7

STATUS_MESSAGES = {
    ERR_INITIAL_MERKLE: "checkInitialTreeProofs: at least one Merkle proof failed",   # Plonk/FRI.hs:108
    ERR_STEP_MERKLE: "folding step Merkle proof does not check out",                  # Plonk/FRI.hs:310
    ERR_STEP_EVAL: "folding step evaluation does not match the opening",              # Plonk/FRI.hs:311
    ERR_STEP_ARITY: "folding stpe: reduction strategy incompatibility",               # Plonk/FRI.hs:312
    ERR_SHAPE: "shape mismatch between proof and circuit",
    ERR_CIRCUIT: "circuit not supported",
    ERR_PARSE: "JSON did not decode",
}

# function return codes
E_OK, E_PARSE, E_CIRCUIT, E_SHAPE, E_ARG, E_DEVICE, E_NODEVICE = 0, -1, -2, -3, -4, -5, -6
# opt-in plonky2 conventions the reference does not implement (include/p2v.h P2V_EXT_*)
EXT_PARAMS_ARITIES, EXT_HIDING, EXT_HASH_OR_NOOP, EXT_PLONKY2 = 1, 2, 4, 7

FLAG_INPUT_DEVICE = 1
FLAG_RESULT_DEVICE = 2
FLAG_NO_SYNC = 4
FLAG_UNIT_FILTERS = 8   # parity mode (tests only): every gate filter / lookup selector := 1
FLAG_INPUT_TILED = 16   # the batch in 64-proof tiles [n/64][words][64] (tile_proofs)
FLAG_LOOKAHEAD = 32     # the device batch is complete at the call: its transcript may run ahead (include/p2v.h)
SHAPE_LIMIT = 1 << 20   # public inputs / final-polynomial coefficients a shape variant may hold (include/p2v.h)
SHAPE_VARIANTS_KEPT = 8   # shape variants a circuit keeps (least recently used evicted)


class P2VError(RuntimeError):
    """A libp2v call failed (return code < 0)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libp2v error {code}: {message}")
        self.code = code
        self.message = message


class VerifierError(RuntimeError):
    """The reference verifier would raise `error` for this proof (status < 0)."""

    def __init__(self, status: int):
        super().__init__(STATUS_MESSAGES.get(status, f"status {status}"))
        self.status = status


class _Info(ctypes.Structure):
    _fields_ = [
        ("degree_bits", ctypes.c_int32), ("lde_bits", ctypes.c_int32), ("cap_height", ctypes.c_int32),
        ("num_challenges", ctypes.c_int32), ("num_query_rounds", ctypes.c_int32), ("num_fri_steps", ctypes.c_int32),
        ("final_poly_len", ctypes.c_int32), ("num_public_inputs", ctypes.c_int32), ("num_openings_this", ctypes.c_int32),
        ("num_openings_next", ctypes.c_int32), ("has_lookups", ctypes.c_int32), ("num_gates", ctypes.c_int32),
        ("proof_words", ctypes.c_int64), ("trace_words", ctypes.c_int64), ("oracle_widths", ctypes.c_int32 * 4),
        ("step_arity_bits", ctypes.c_int32 * 8), ("leaf_widths", ctypes.c_int32 * 4), ("ext", ctypes.c_uint32),
    ]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libp2v.so (built in-tree by `make -C plonky2-verifier_amd`).  Fails loudly."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `make -C {_HERE}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u64p, i8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p
    L.p2v_circuit_from_json.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(vp)]
    L.p2v_circuit_free.argtypes = [vp]
    L.p2v_circuit_free.restype = None
    L.p2v_circuit_get_info.argtypes = [vp, ctypes.POINTER(_Info)]
    L.p2v_pack_proof_json.argtypes = [vp, ctypes.c_char_p, sz, u64p]
    L.p2v_pack_proofs_json.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), sz, u64p, vp, ctypes.c_int]
    L.p2v_circuit_from_words.argtypes = [u64p, sz, ctypes.POINTER(vp)]
    L.p2v_circuit_from_json_ex.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.p2v_circuit_from_words_ex.argtypes = [u64p, sz, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.p2v_pack_proof_words.argtypes = [vp, u64p, sz, u64p]
    L.p2v_pack_proof_bytes.argtypes = [vp, ctypes.c_char_p, sz, u64p]
    L.p2v_tiled_words.argtypes = [sz, sz]
    L.p2v_tiled_words.restype = sz
    L.p2v_tile_proofs.argtypes = [u64p, sz, sz, u64p]
    L.p2v_tile_proofs.restype = None
    L.p2v_device_count.argtypes = []
    L.p2v_verifier_create.argtypes = [vp, ctypes.c_int, sz, ctypes.POINTER(vp)]
    L.p2v_verifier_free.argtypes = [vp]
    L.p2v_verifier_free.restype = None
    L.p2v_verifier_run.argtypes = [vp, u64p, sz, i8p, u64p, vp, ctypes.c_uint32]
    L.p2v_verifier_chain.argtypes = [vp, vp]
    L.p2v_verifier_run_json.argtypes = [vp, vp, vp, sz, i8p, vp, vp, vp]
    L.p2v_verifier_pack_json.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp]
    L.p2v_verifier_run_bytes.argtypes = [vp, vp, vp, sz, i8p, vp, vp, vp]
    L.p2v_verifier_pack_bytes.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp]
    L.p2v_verify_batch.argtypes = [vp, u64p, sz, i8p, ctypes.c_int]
    L.p2v_verify_batch_devices.argtypes = [vp, u64p, sz, i8p, ctypes.POINTER(ctypes.c_int), ctypes.c_int, sz]
    L.p2v_verify_batch_bytes.argtypes = [vp, vp, vp, sz, i8p, vp, vp, ctypes.c_int, sz]
    L.p2v_verifier_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    L.p2v_selftest.argtypes = [ctypes.c_int, ctypes.c_int, u64p, u64p, u64p, sz]
    L.p2v_count_mismatches.argtypes = [i8p, i8p, sz, u64p, vp]
    L.p2v_clock_probe.argtypes = [u64p, ctypes.c_int, vp]
    L.p2v_proof_shape_json.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.p2v_proof_shape_words.argtypes = [u64p, sz, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.p2v_circuit_shape_variant.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.p2v_kernel_names.restype = ctypes.c_char_p
    L.p2v_last_error_message.restype = ctypes.c_char_p
    L.p2v_version.restype = ctypes.c_char_p
    _lib = L
    return L


def build_info() -> dict:
    """The loaded library's version string and source hash (p2v_version, csrc/version.cpp) next to
    the hash of the sources in this tree (srchash.py), and whether they agree."""
    import srchash
    v = lib().p2v_version().decode()
    built = v.rsplit(" src ", 1)[1] if " src " in v else "unknown"
    tree = srchash.source_hash(_HERE)
    return {"version": v, "lib": os.path.abspath(LIB_PATH), "src_hash_built": built, "src_hash_tree": tree,
            "match": built == tree}


def check_build() -> dict:
    """Refuse a libp2v.so built from other sources than the tree this process runs from
    (VERDICT r5 item 5).  P2V_LIB builds (A/B measurement variants) are exempt: reported only."""
    info = build_info()
    if not info["match"] and not os.environ.get("P2V_LIB"):
        raise ImportError(f"{info['lib']} was built from sources {info['src_hash_built']}, the tree holds "
                          f"{info['src_hash_tree']}: rebuild with `make -C {_HERE}`")
    return info


def _check(rc: int) -> None:
    if rc != E_OK:
        raise P2VError(rc, lib().p2v_last_error_message().decode(errors="replace"))


def _bytes(x: Union[str, bytes]) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


@dataclass(frozen=True)
class CircuitInfo:
    degree_bits: int
    lde_bits: int
    cap_height: int
    num_challenges: int
    num_query_rounds: int
    num_fri_steps: int
    final_poly_len: int
    num_public_inputs: int
    num_openings_this: int
    num_openings_next: int
    has_lookups: bool
    num_gates: int
    proof_words: int
    trace_words: int
    oracle_widths: tuple
    step_arity_bits: tuple
    leaf_widths: tuple = ()
    ext: int = 0


class VerifierCircuitData:
    """VerifierCircuitData = VerifierOnlyCircuitData + CommonCircuitData (Types.hs:220-224).

    Decoding and every circuit-level check of the reference (unknown gate, selector
    tally, unsupported reduction strategy, ...) happen once here (P2VError otherwise)."""

    def __init__(self, handle: int):
        self._h = ctypes.c_void_p(handle)
        inf = _Info()
        _check(lib().p2v_circuit_get_info(self._h, ctypes.byref(inf)))
        self.info = CircuitInfo(
            inf.degree_bits, inf.lde_bits, inf.cap_height, inf.num_challenges, inf.num_query_rounds, inf.num_fri_steps,
            inf.final_poly_len, inf.num_public_inputs, inf.num_openings_this, inf.num_openings_next, bool(inf.has_lookups),
            inf.num_gates, inf.proof_words, inf.trace_words, tuple(inf.oracle_widths), tuple(inf.step_arity_bits[: inf.num_fri_steps]),
            tuple(inf.leaf_widths), inf.ext)

    @classmethod
    def from_json(cls, common_json: Union[str, bytes], vkey_json: Union[str, bytes], ext: int = 0) -> "VerifierCircuitData":
        """ext: opt-in plonky2 conventions the reference lacks (EXT_* below, include/p2v.h);
        0 = exactly the reference's semantics."""
        c, v = _bytes(common_json), _bytes(vkey_json)
        h = ctypes.c_void_p()
        _check(lib().p2v_circuit_from_json_ex(c, len(c), v, len(v), ext, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def from_words(cls, words: np.ndarray, ext: int = 0) -> "VerifierCircuitData":
        """The word-encoded Types.hs value (include/p2v.h; what the Haskell shim marshals)."""
        w = np.ascontiguousarray(words, dtype=np.uint64)
        h = ctypes.c_void_p()
        _check(lib().p2v_circuit_from_words_ex(w.ctypes.data, w.size, ext, ctypes.byref(h)))
        return cls(h.value)

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def shape_variant(self, num_public_inputs: int, final_poly_len: int) -> "VerifierCircuitData":
        """The same circuit with a packed layout for these public-input / final-polynomial
        lengths (p2v_circuit_shape_variant); self when they are the circuit's own."""
        if (num_public_inputs, final_poly_len) == (self.info.num_public_inputs, self.info.final_poly_len):
            return self
        # the most recently used variants: a variant's handle owns pooled device
        # pipelines once it has verified, so proofs of many distinct lengths must not grow device
        # memory without bound; an evicted variant is freed when its last user drops it
        from collections import OrderedDict
        cache = self.__dict__.setdefault("_variants", OrderedDict())
        key = (num_public_inputs, final_poly_len)
        if key in cache:
            cache.move_to_end(key)
        else:
            h = ctypes.c_void_p()
            _check(lib().p2v_circuit_shape_variant(self._h, num_public_inputs, final_poly_len, ctypes.byref(h)))
            cache[key] = VerifierCircuitData(h.value)
            while len(cache) > SHAPE_VARIANTS_KEPT:
                cache.popitem(last=False)
        return cache[key]

    def for_proof(self, proof_json: Union[str, bytes]) -> "VerifierCircuitData":
        """The circuit (or its shape variant) whose layout holds this proof's public inputs and
        final polynomial as given (the reference reads both at any length)."""
        b = _bytes(proof_json)
        npi, nf = ctypes.c_int(), ctypes.c_int()
        if lib().p2v_proof_shape_json(b, len(b), ctypes.byref(npi), ctypes.byref(nf)) != E_OK:
            return self   # undecodable: packing reports it
        return self.shape_variant(npi.value, nf.value)

    def for_proof_words(self, words: np.ndarray) -> "VerifierCircuitData":
        """for_proof for a word-encoded ProofWithPublicInputs (include/p2v.h)."""
        w = np.ascontiguousarray(words, dtype=np.uint64)
        npi, nf = ctypes.c_int(), ctypes.c_int()
        if lib().p2v_proof_shape_words(w.ctypes.data, w.size, ctypes.byref(npi), ctypes.byref(nf)) != E_OK:
            return self
        return self.shape_variant(npi.value, nf.value)

    def pack_words(self, words: np.ndarray, out: Optional[np.ndarray] = None) -> np.ndarray:
        """A word-encoded ProofWithPublicInputs (include/p2v.h) -> packed u64 words."""
        w = np.ascontiguousarray(words, dtype=np.uint64)
        if out is None:
            out = np.empty(self.info.proof_words, dtype=np.uint64)
        assert out.dtype == np.uint64 and out.size == self.info.proof_words and out.flags.c_contiguous
        _check(lib().p2v_pack_proof_words(self._h, w.ctypes.data, w.size, out.ctypes.data))
        return out

    def pack_bytes(self, data: bytes, out: Optional[np.ndarray] = None) -> np.ndarray:
        """plonky2's binary ProofWithPublicInputs serialization (include/p2v.h
        p2v_pack_proof_bytes) -> packed u64 words of this circuit."""
        b = bytes(data)
        if out is None:
            out = np.empty(self.info.proof_words, dtype=np.uint64)
        assert out.dtype == np.uint64 and out.size == self.info.proof_words and out.flags.c_contiguous
        _check(lib().p2v_pack_proof_bytes(self._h, b, len(b), out.ctypes.data))
        return out

    def pack(self, proof_json: Union[str, bytes], out: Optional[np.ndarray] = None) -> np.ndarray:
        """ProofWithPublicInputs JSON (Types.hs:245-254) -> packed u64 words of this circuit."""
        b = _bytes(proof_json)
        if out is None:
            out = np.empty(self.info.proof_words, dtype=np.uint64)
        assert out.dtype == np.uint64 and out.size == self.info.proof_words and out.flags.c_contiguous
        _check(lib().p2v_pack_proof_json(self._h, b, len(b), out.ctypes.data))
        return out

    def pack_many(self, proofs: Sequence[Union[str, bytes]], threads: int = 0, codes: Optional[np.ndarray] = None) -> np.ndarray:
        """A list of ProofWithPublicInputs JSON texts -> [n, proof_words] packed words, on
        `threads` host threads (0: all cores; p2v_pack_proofs_json).  Raises P2VError for the
        first proof that does not decode unless `codes` (int32 [n]) is given to receive the
        per-proof codes (rows of failed proofs are then undefined)."""
        bs = [_bytes(p) for p in proofs]
        n = len(bs)
        arr = np.empty((n, self.info.proof_words), dtype=np.uint64)
        if n == 0:
            return arr
        ptrs = (ctypes.c_char_p * n)(*bs)
        lens = (ctypes.c_size_t * n)(*[len(b) for b in bs])
        cd = np.empty(n, dtype=np.int32) if codes is None else codes
        assert cd.dtype == np.int32 and cd.size == n
        nfail = lib().p2v_pack_proofs_json(self._h, ptrs, lens, n, arr.ctypes.data, cd.ctypes.data, threads)
        if nfail < 0 or (nfail > 0 and codes is None):
            bad = int(np.flatnonzero(cd != E_OK)[0]) if nfail > 0 else 0
            raise P2VError(int(cd[bad]) if nfail > 0 else nfail, lib().p2v_last_error_message().decode(errors="replace"))
        return arr

    def __del__(self):
        try:
            if getattr(self, "_h", None) and self._h.value:
                lib().p2v_circuit_free(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


@dataclass
class ProofWithPublicInputs:
    """ProofWithPublicInputs (Types.hs:245-254), kept as JSON text until packed."""

    json: bytes

    @classmethod
    def from_json(cls, text: Union[str, bytes]) -> "ProofWithPublicInputs":
        return cls(_bytes(text))


def device_count() -> int:
    return int(lib().p2v_device_count())


class BatchVerifier:
    """A per-device workspace bound to one circuit (all device memory allocated here)."""

    def __init__(self, circuit: VerifierCircuitData, device: int = 0, max_batch: int = 4096):
        self.circuit = circuit
        self.device = device
        self.max_batch = max_batch
        h = ctypes.c_void_p()
        _check(lib().p2v_verifier_create(circuit.handle, device, max_batch, ctypes.byref(h)))
        self._h = h

    def run(self, proofs: np.ndarray, trace: bool = False, unit_filters: bool = False, stream: int = 0,
            tiled: bool = False):
        """proofs: uint64 [n, proof_words] host array.  Returns int8 statuses (and trace).
        unit_filters: parity mode (P2V_FLAG_UNIT_FILTERS), statuses meaningless.  stream: a
        hipStream_t handle (0: the default stream).  tiled: the batch goes to the device in the
        64-proof tiled layout (P2V_FLAG_INPUT_TILED; tiled here with tile_proofs)."""
        proofs = np.ascontiguousarray(proofs, dtype=np.uint64)
        n = proofs.shape[0]
        src = tile_proofs(proofs) if tiled else proofs
        res = np.empty(n, dtype=np.int8)
        tr = np.empty((n, self.circuit.info.trace_words), dtype=np.uint64) if trace else None
        flags = (FLAG_UNIT_FILTERS if unit_filters else 0) | (FLAG_INPUT_TILED if tiled else 0)
        _check(lib().p2v_verifier_run(self._h, src.ctypes.data, n, res.ctypes.data,
                                      tr.ctypes.data if trace else None, ctypes.c_void_p(stream) if stream else None, flags))
        return (res, tr) if trace else res

    @staticmethod
    def _json_batch(proofs):
        if isinstance(proofs, tuple):
            blob, offs = proofs
            blob = np.ascontiguousarray(blob, dtype=np.uint8) if not isinstance(blob, np.ndarray) else blob
            return blob, np.ascontiguousarray(offs, dtype=np.uint64)
        bs = [_bytes(p) for p in proofs]
        offs = np.zeros(len(bs) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(b) for b in bs])
        return np.frombuffer(b"".join(bs), dtype=np.uint8), offs

    def run_json(self, proofs: Union[Sequence[Union[str, bytes]], tuple], stream: int = 0):
        """JSON texts -> (int8 statuses, int32 decode codes) via p2v_verifier_run_json (texts
        copied to the device and packed there).  `proofs` is a list of texts, or a pair
        (uint8 blob array, uint64 offsets[n + 1]) e.g. in pinned memory.  How many proofs the
        device packer took (the rest went through the host reader) is left in
        `self.last_json_device`."""
        blob, offs = self._json_batch(proofs)
        n = offs.size - 1
        res = np.empty(n, dtype=np.int8)
        codes = np.empty(n, dtype=np.int32)
        ndev = ctypes.c_size_t(0)
        _check(lib().p2v_verifier_run_json(self._h, blob.ctypes.data, offs.ctypes.data, n, res.ctypes.data, codes.ctypes.data,
                                           ctypes.addressof(ndev), ctypes.c_void_p(stream)))
        self.last_json_device = ndev.value
        return res, codes

    def pack_json(self, proofs: Union[Sequence[Union[str, bytes]], tuple], stream: int = 0):
        """JSON texts -> (uint64 [n, proof_words] packed words, int32 decode codes), packed on
        the device (p2v_verifier_pack_json); same inputs as run_json."""
        blob, offs = self._json_batch(proofs)
        n = offs.size - 1
        words = np.empty((n, self.circuit.info.proof_words), dtype=np.uint64)
        codes = np.empty(n, dtype=np.int32)
        ndev = ctypes.c_size_t(0)
        _check(lib().p2v_verifier_pack_json(self._h, blob.ctypes.data, offs.ctypes.data, n, codes.ctypes.data,
                                            ctypes.addressof(ndev), words.ctypes.data, ctypes.c_void_p(stream)))
        self.last_json_device = ndev.value
        return words, codes

    def run_bytes(self, proofs: Union[Sequence[bytes], tuple], stream: int = 0):
        """plonky2 binary proofs (p2v_pack_proof_bytes' format) -> (int8 statuses, int32 decode
        codes) via p2v_verifier_run_bytes (copied to the device and packed there).  Same inputs as
        run_json; the device-packed count is left in `self.last_bytes_device`."""
        blob, offs = self._json_batch(proofs)
        n = offs.size - 1
        res = np.empty(n, dtype=np.int8)
        codes = np.empty(n, dtype=np.int32)
        ndev = ctypes.c_size_t(0)
        _check(lib().p2v_verifier_run_bytes(self._h, blob.ctypes.data, offs.ctypes.data, n, res.ctypes.data, codes.ctypes.data,
                                            ctypes.addressof(ndev), ctypes.c_void_p(stream)))
        self.last_bytes_device = ndev.value
        return res, codes

    def pack_bytes(self, proofs: Union[Sequence[bytes], tuple], stream: int = 0):
        """plonky2 binary proofs -> (uint64 [n, proof_words] packed words, int32 decode codes),
        packed on the device (p2v_verifier_pack_bytes)."""
        blob, offs = self._json_batch(proofs)
        n = offs.size - 1
        words = np.empty((n, self.circuit.info.proof_words), dtype=np.uint64)
        codes = np.empty(n, dtype=np.int32)
        ndev = ctypes.c_size_t(0)
        _check(lib().p2v_verifier_pack_bytes(self._h, blob.ctypes.data, offs.ctypes.data, n, codes.ctypes.data,
                                             ctypes.addressof(ndev), words.ctypes.data, ctypes.c_void_p(stream)))
        self.last_bytes_device = ndev.value
        return words, codes

    def run_device(self, proofs_ptr: int, n: int, results_ptr: int, stream: int = 0, trace_ptr: int = 0,
                   sync: bool = True, tiled: bool = False, lookahead: bool = False) -> None:
        """Device-resident batch: raw device pointers (e.g. torch tensor .data_ptr()) and a
        hipStream_t handle (torch.cuda.current_stream().cuda_stream).  tiled: the batch is in the
        64-proof tiled layout (P2V_FLAG_INPUT_TILED, tile_proofs).  lookahead: the batch is already
        complete in device memory, so its transcript may run ahead of this workspace's earlier
        batches (P2V_FLAG_LOOKAHEAD)."""
        flags = (FLAG_INPUT_DEVICE | FLAG_RESULT_DEVICE | (0 if sync else FLAG_NO_SYNC) | (FLAG_INPUT_TILED if tiled else 0)
                 | (FLAG_LOOKAHEAD if lookahead else 0))
        _check(lib().p2v_verifier_run(self._h, ctypes.c_void_p(proofs_ptr), n, ctypes.c_void_p(results_ptr),
                                      ctypes.c_void_p(trace_ptr) if trace_ptr else None, ctypes.c_void_p(stream), flags))

    def last_timings(self) -> dict:
        buf = (ctypes.c_float * 16)()
        k = lib().p2v_verifier_last_timings(self._h, buf, 16)
        names = lib().p2v_kernel_names().decode().split(",")
        return {names[i]: float(buf[i]) for i in range(k) if buf[i] > 0}   # 0: kernel not launched in this build

    def chain(self, prev: Optional["BatchVerifier"]) -> None:
        """p2v_verifier_chain: later runs of this workspace start phase 1 after `prev`'s latest
        phase 1 (staggered workspaces; results unaffected).  prev=None unlinks.  Keeps a
        reference to prev so it outlives the link."""
        _check(lib().p2v_verifier_chain(self._h, prev._h if prev is not None else None))
        self._chain_prev = prev

    def __del__(self):
        try:
            if getattr(self, "_h", None) and self._h.value:
                lib().p2v_verifier_free(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def tile_proofs(packed: np.ndarray) -> np.ndarray:
    """Proof-major packed rows [n, proof_words] -> the 64-proof tiled layout of
    P2V_FLAG_INPUT_TILED (include/p2v.h): ceil(n/64) tiles of [proof_words][64], padded with 0.
    Flat uint64 array of p2v_tiled_words(n, proof_words) words."""
    packed = np.ascontiguousarray(packed, dtype=np.uint64)
    n, W = packed.shape
    t = (n + 63) // 64
    pad = np.zeros((t * 64, W), dtype=np.uint64)
    pad[:n] = packed
    return np.ascontiguousarray(pad.reshape(t, 64, W).transpose(0, 2, 1)).reshape(-1)


# ----------------------------------------------------------------------------- intermediates
# The reference's driver (src/testmain.hs:54-63) prints the sub-results of verifyProof:
# proofChallenges, evalCombinedPlonkConstraints and checkCombinedPlonkEquations'.  The same values,
# computed by the GPU kernels of the batch path, come out of libp2v's per-proof trace
# (include/p2v.h "debug trace layout"); these mirror those functions.
FExt = tuple   # (re, im), GoldilocksExt.hs:24-32


def trace_offsets(r: int, S: int, Q: int) -> dict:
    """Word offsets of the per-proof trace (include/p2v.h)."""
    o = {"pi_hash": 0, "betas": 4}
    o["gammas"] = o["betas"] + r
    o["alphas"] = o["gammas"] + r
    o["deltas"] = o["alphas"] + r
    o["zeta"] = o["deltas"] + 4 * r
    o["fri_alpha"] = o["zeta"] + 2
    o["fri_betas"] = o["fri_alpha"] + 2
    o["pow"] = o["fri_betas"] + 2 * S
    o["query_idx"] = o["pow"] + 1
    o["combined"] = o["query_idx"] + Q
    o["quotient"] = o["combined"] + 2 * r
    o["q_initial"] = o["quotient"] + 2 * r
    o["q_folded"] = o["q_initial"] + 2 * Q
    o["q_final"] = o["q_folded"] + 2 * Q
    o["flags"] = o["q_final"] + 2 * Q
    o["lut_re"] = o["flags"] + 1
    return o


@dataclass(frozen=True)
class FriChallenges:   # Challenge/FRI.hs:24-30
    fri_alpha: FExt
    fri_betas: tuple
    fri_pow_response: int
    fri_query_indices: tuple


@dataclass(frozen=True)
class ProofChallenges:   # Challenge/Verifier.hs:45-53
    plonk_betas: tuple
    plonk_gammas: tuple
    plonk_alphas: tuple
    plonk_deltas: tuple      # per round (A, B, alpha, delta) = chunksOf 4 (betas ++ gammas ++ new), :36-40; () without lookups
    plonk_zeta: FExt
    fri_challenges: FriChallenges
    public_inputs_hash: tuple


def _trace_one(vkey: VerifierCircuitData, proof, device: int) -> np.ndarray:
    text = proof.json if isinstance(proof, ProofWithPublicInputs) else _bytes(proof)
    bv = BatchVerifier(vkey, device, 1)
    _res, tr = bv.run(vkey.pack(text)[None, :], trace=True)
    return tr[0]


def _ext(tr, o) -> FExt:
    return (int(tr[o]), int(tr[o + 1]))


def proof_challenges(vkey: VerifierCircuitData, proof, device: int = 0) -> ProofChallenges:
    """proofChallenges (Challenge/Verifier.hs:58-103): the Fiat-Shamir challenges of one proof,
    as the GPU transcript derives them."""
    inf = vkey.info
    r, S, Q = inf.num_challenges, inf.num_fri_steps, inf.num_query_rounds
    tr, o = _trace_one(vkey, proof, device), trace_offsets(r, S, Q)
    rng = lambda k, n: tuple(int(x) for x in tr[o[k]: o[k] + n])   # noqa: E731
    deltas = tuple(rng("deltas", 4 * r)[4 * i: 4 * i + 4] for i in range(r)) if inf.has_lookups else ()
    fri = FriChallenges(_ext(tr, o["fri_alpha"]), tuple(_ext(tr, o["fri_betas"] + 2 * i) for i in range(S)),
                        int(tr[o["pow"]]), rng("query_idx", Q))
    return ProofChallenges(rng("betas", r), rng("gammas", r), rng("alphas", r), deltas, _ext(tr, o["zeta"]), fri,
                           rng("pi_hash", 4))


def eval_combined_plonk_constraints(vkey: VerifierCircuitData, proof, device: int = 0) -> List[FExt]:
    """evalCombinedPlonkConstraints (Plonk/Vanishing.hs:48-51): the vanishing terms at zeta
    combined with powers of each round's alpha, one F^2 value per challenge round."""
    inf = vkey.info
    r = inf.num_challenges
    tr, o = _trace_one(vkey, proof, device), trace_offsets(r, inf.num_fri_steps, inf.num_query_rounds)
    return [_ext(tr, o["combined"] + 2 * i) for i in range(r)]


def check_combined_plonk_equations(vkey: VerifierCircuitData, proof, device: int = 0) -> bool:
    """checkCombinedPlonkEquations' (Plonk/Verifier.hs:35-51): the quotient identity
    Q_i(zeta) (zeta^n - 1) == C_i(zeta) for every challenge round (eqs_ok of verifyProof)."""
    inf = vkey.info
    tr, o = _trace_one(vkey, proof, device), trace_offsets(inf.num_challenges, inf.num_fri_steps, inf.num_query_rounds)
    return bool(int(tr[o["flags"]]) & 1)


def _status_to_bool(st: int) -> bool:
    if st == ACCEPT:
        return True
    if st == REJECT:
        return False
    raise VerifierError(int(st))


def device_selftest(op: int, a: np.ndarray, b: Optional[np.ndarray] = None, device: int = 0) -> np.ndarray:
    """p2v_selftest (include/p2v.h): the device field multiply (op 0, a * b mod p; op 3 the S-box's
    form), Poseidon permutation (op 1, a = [n, 12] states), 2-to-1 compression form (op 2, words
    8..11 taken as 0, words 0..3 returned), one MDS layer (op 4), the S-box forms (ops 5-8, x^7;
    op 6 the grouped pair (a[i], b[i]) -> out [n, 2]) and the latency forms of the permutation
    (ops 9-11: row, quad, pair) on `device`."""
    a = np.ascontiguousarray(a, dtype=np.uint64)
    n = a.shape[0]
    out = np.zeros((n, 2), dtype=np.uint64) if op == 6 else np.zeros_like(a)   # op 4: b = [kl[12], kh[12]]
    bb = np.ascontiguousarray(b, dtype=np.uint64) if b is not None else None
    _check(lib().p2v_selftest(device, op, a.ctypes.data, bb.ctypes.data if bb is not None else None, out.ctypes.data, n))
    return out


def count_mismatches(results_ptr: int, expect_ptr: int, n: int, counters_ptr: int, stream: int = 0) -> None:
    """p2v_count_mismatches (device pointers, enqueued on `stream`): counters[0] += #{results !=
    expect}, counters[1] += 1.  The bench folds every timed launch's statuses into it."""
    _check(lib().p2v_count_mismatches(ctypes.c_void_p(results_ptr), ctypes.c_void_p(expect_ptr), n,
                                      ctypes.c_void_p(counters_ptr), ctypes.c_void_p(stream)))


def clock_probe(stamps_ptr: int, nblocks: int, stream: int = 0) -> None:
    """p2v_clock_probe: nblocks one-wave workgroups write (XCC id, s_memtime, s_memrealtime) to
    the device buffer stamps[3 * nblocks] (u64), on `stream`."""
    _check(lib().p2v_clock_probe(ctypes.c_void_p(stamps_ptr), nblocks, ctypes.c_void_p(stream)))


def clock_from_probes(start: np.ndarray, end: np.ndarray) -> Optional[dict]:
    """The shader clock over the interval between two clock_probe launches: per XCD, the median
    stamp of each probe, d(s_memtime) / d(s_memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS
    item 6).  start / end: [nblocks, 3] u64 stamps."""
    per = {}
    for x in sorted(set(int(v) for v in start[:, 0]) & set(int(v) for v in end[:, 0])):
        a, b = start[start[:, 0] == x], end[end[:, 0] == x]
        dt = float(np.median(b[:, 1].astype(np.float64))) - float(np.median(a[:, 1].astype(np.float64)))
        dr = float(np.median(b[:, 2].astype(np.float64))) - float(np.median(a[:, 2].astype(np.float64)))
        if dr > 0:
            per[x] = dt / dr * 0.1   # GHz: memrealtime counts at 100 MHz
    if not per:
        return None
    v = list(per.values())
    return {"clock_ghz": round(float(np.mean(v)), 4), "min_ghz": round(min(v), 4), "max_ghz": round(max(v), 4),
            "xcds": len(per), "interval_ms": round(dr / 1e5, 3)}


def verify_proof(vkey: VerifierCircuitData, proof: Union[ProofWithPublicInputs, str, bytes], device: int = 0) -> bool:
    """verifyProof (Plonk/Verifier.hs:56-65): True / False, or VerifierError where the
    reference raises `error`.  Public inputs and the final polynomial are taken at the length
    the proof carries (a shape variant of the circuit when it differs, as the reference does)."""
    text = proof.json if isinstance(proof, ProofWithPublicInputs) else _bytes(proof)
    vk = vkey
    packed = np.empty((1, vkey.info.proof_words), dtype=np.uint64)
    rc = lib().p2v_pack_proof_json(vkey.handle, text, len(text), packed.ctypes.data)
    if rc == E_SHAPE:   # other public-input / final-polynomial lengths: the circuit's shape variant
        vk = vkey.for_proof(text)
        packed = vk.pack(text)[None, :]
    else:
        _check(rc)
    res = np.empty(1, dtype=np.int8)
    # libp2v keeps the circuit's verifier between calls (p2v_verify_batch's pool), so a repeated
    # call costs the kernels, not a workspace
    _check(lib().p2v_verify_batch(vk.handle, packed.ctypes.data, 1, res.ctypes.data, device))
    return _status_to_bool(int(res[0]))


def _pack_error(vkey: VerifierCircuitData, text: bytes) -> str:
    """The host packer's message for one proof that does not pack against `vkey`."""
    out = np.empty(vkey.info.proof_words, dtype=np.uint64)
    rc = lib().p2v_pack_proof_json(vkey.handle, text, len(text), out.ctypes.data)
    return lib().p2v_last_error_message().decode(errors="replace") if rc != E_OK else "ok"


def verify_proof_batch(vkey: VerifierCircuitData, proofs: Iterable[Union[ProofWithPublicInputs, str, bytes]],
                       device: int = 0) -> List[Union[bool, VerifierError]]:
    """Batch form: one entry per proof, True/False or the VerifierError the reference would raise.
    Proofs whose public-input / final-polynomial lengths differ from the circuit's are verified in
    sub-batches of their shape variant."""
    texts = [p.json if isinstance(p, ProofWithPublicInputs) else _bytes(p) for p in proofs]
    if not texts:
        return []
    n = len(texts)
    res = np.empty(n, dtype=np.int8)
    # one pass against the circuit itself; only proofs whose lengths differ (E_SHAPE) are
    # re-read for their shape and packed again against that shape variant
    codes = np.empty(n, dtype=np.int32)
    packed = vkey.pack_many(texts, codes=codes)
    groups = {}
    for i in np.flatnonzero(codes != E_OK):
        if codes[i] != E_SHAPE:
            raise P2VError(int(codes[i]), f"proof {i}: " + _pack_error(vkey, texts[i]))
        try:
            vk = vkey.for_proof(texts[i])
        except P2VError:
            # lengths past this build's limits (include/p2v.h, 2^20): the transcript cannot match
            # the circuit's, so the reference's answer is False (barring a PoW collision).  Any
            # other shape-variant failure (a circuit that does not validate, allocation) is an
            # error, not a verdict
            npi, nf = ctypes.c_int(), ctypes.c_int()
            b = texts[i]
            if (lib().p2v_proof_shape_json(b, len(b), ctypes.byref(npi), ctypes.byref(nf)) == E_OK
                    and (npi.value > SHAPE_LIMIT or nf.value > SHAPE_LIMIT)):
                res[i] = REJECT
                continue
            raise
        if vk is vkey:   # another list-length mismatch: an `error` in the reference as well
            raise P2VError(E_SHAPE, f"proof {i}: " + _pack_error(vkey, texts[i]))
        groups.setdefault(id(vk), (vk, []))[1].append(int(i))
    good = np.flatnonzero(codes == E_OK)
    if good.size:
        sub = np.empty(good.size, dtype=np.int8)
        rows = np.ascontiguousarray(packed[good])
        _check(lib().p2v_verify_batch(vkey.handle, rows.ctypes.data, good.size, sub.ctypes.data, device))
        res[good] = sub
    for vk, idx in groups.values():
        rows = vk.pack_many([texts[i] for i in idx])
        sub = np.empty(len(idx), dtype=np.int8)
        _check(lib().p2v_verify_batch(vk.handle, rows.ctypes.data, len(idx), sub.ctypes.data, device))
        res[idx] = sub
    out: List[Union[bool, VerifierError]] = []
    for st in res:
        out.append(True if st == ACCEPT else False if st == REJECT else VerifierError(int(st)))
    return out


# ----------------------------------------------------------------------------- multi-GPU
def verify_batch_devices(vkey: VerifierCircuitData, packed: np.ndarray, devices: Sequence[int], chunk: int = 0) -> np.ndarray:
    """Single-process multi-GPU verification (p2v_verify_batch_devices): contiguous shards of
    the packed batch, one per entry of `devices`, each on its own host thread; int8 statuses."""
    packed = np.ascontiguousarray(packed, dtype=np.uint64)
    n = packed.shape[0]
    res = np.empty(n, dtype=np.int8)
    devs = (ctypes.c_int * len(devices))(*devices)
    _check(lib().p2v_verify_batch_devices(vkey.handle, packed.ctypes.data, n, res.ctypes.data, devs, len(devices), chunk))
    return res


def verify_batch(vkey: VerifierCircuitData, packed: np.ndarray, device: int = 0) -> np.ndarray:
    """p2v_verify_batch: packed rows [n, proof_words] in host memory (pinned for the full link
    rate), verified by the circuit's pooled verifier on `device`, H2D copies overlapped with the
    verification in chunks; int8 statuses."""
    packed = np.ascontiguousarray(packed, dtype=np.uint64)
    n = packed.shape[0]
    res = np.empty(n, dtype=np.int8)
    _check(lib().p2v_verify_batch(vkey.handle, packed.ctypes.data, n, res.ctypes.data, device))
    return res


def verify_batch_bytes(vkey: VerifierCircuitData, proofs: Union[Sequence[bytes], tuple], device: int = 0, chunk: int = 0):
    """p2v_verify_batch_bytes: plonky2 binary proofs (a list, or a (uint8 blob, uint64 offsets[n+1])
    pair, e.g. in pinned memory) -> (int8 statuses, int32 decode codes, proofs the device packed)."""
    blob, offs = BatchVerifier._json_batch(proofs)
    n = offs.size - 1
    res = np.empty(n, dtype=np.int8)
    codes = np.empty(n, dtype=np.int32)
    ndev = ctypes.c_size_t(0)
    _check(lib().p2v_verify_batch_bytes(vkey.handle, blob.ctypes.data, offs.ctypes.data, n, res.ctypes.data, codes.ctypes.data,
                                        ctypes.addressof(ndev), device, chunk))
    return res, codes, ndev.value


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous near-equal shard [start, end) of n proofs for `rank` of `world`.
    Proofs are independent (verifyProof has no cross-proof state), so a batch shards
    across GPUs with no collective on the data path."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def verify_sharded(vkey: VerifierCircuitData, packed: np.ndarray, rank: int, world: int, device: int,
                   group=None, verify_shard=None, gather_group=None) -> np.ndarray:
    """Each rank verifies its shard of `packed` on its own GPU; the int8 statuses are then
    gathered so every rank holds the full result vector (one all_gather of the padded int8
    shards, the only cross-rank traffic; on the RCCL backend the gather runs on the device).
    gather_group: a gloo group (dist.new_group(backend="gloo")) to gather over instead, on CPU
    tensors -- the fallback when the RCCL path is unavailable or unwanted.
    verify_shard(rows, start, end) -> int8 statuses replaces the rank's BatchVerifier (tests
    inject a CPU verifier to run the sharding with gloo and no GPU)."""
    s, e = shard_bounds(packed.shape[0], world, rank)
    if verify_shard is None:
        def verify_shard(rows, start, end):
            return BatchVerifier(vkey, device, max(1, end - start)).run(rows)
    local = np.asarray(verify_shard(packed[s:e], s, e), dtype=np.int8) if e > s else np.empty(0, np.int8)
    if world == 1:
        return local
    import torch
    import torch.distributed as dist
    longest = shard_bounds(packed.shape[0], world, 0)[1]   # shard 0 is a longest one
    if gather_group is not None:
        group = gather_group
    dev = torch.device("cuda", device) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    mine = torch.zeros(max(1, longest), dtype=torch.int8, device=dev)
    mine[: len(local)] = torch.from_numpy(local).to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    out = []
    for r in range(world):
        rs, re_ = shard_bounds(packed.shape[0], world, r)
        out.append(parts[r][: re_ - rs].cpu().numpy())
    return np.concatenate(out).astype(np.int8)


# ----------------------------------------------------------------------------- word encoding
# The typed-host form of the boundary (include/p2v.h "word-encoded Types.hs values"): what the
# Haskell shim (bindings/haskell/Plonk/VerifierGPU.hs) marshals from decoded values.  These
# functions derive the same words from the JSON files, following Types.hs field order and the
# Gate/Parser.hs grammar, so tests can hold the words path against the JSON path.
P = 0xFFFFFFFF00000001   # Goldilocks modulus (Algebra/Goldilocks.hs)
WORDS_CIRCUIT_MAGIC = 0x5032564300000001
WORDS_PROOF_MAGIC = 0x5032565000000001
_M64 = (1 << 64) - 1

_GATE_RE = [   # (tag, regex) in Gate/Parser.hs order of alternatives; groups = Int fields
    (0, r"ArithmeticGate \{ num_ops: (\d+) \}$"),
    (1, r"ArithmeticExtensionGate \{ num_ops: (\d+) \}$"),
    (2, r"BaseSumGate \{ num_limbs: (\d+) \} \+ Base: (\d+)$"),
    (3, r"CosetInterpolationGate \{ subgroup_bits: (\d+), degree: (\d+), barycentric_weights: \[([0-9, ]*)\], "
        r"_phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField> \}<D=2>$"),
    (4, r"ConstantGate \{ num_consts: (\d+) \}"),
    (5, r"ExponentiationGate \{ num_power_bits: (\d+) \}"),
    (6, r"LookupGate \{ num_slots: (\d+), lut_hash: \[([0-9, ]*)\] \}"),
    (7, r"LookupTableGate \{ num_slots: (\d+), lut_hash: \[([0-9, ]*)\], last_lut_row: (\d+) \}"),
    (8, r"MulExtensionGate \{ num_ops: (\d+) \}"),
    (9, r"NoopGate"),
    (10, r"PublicInputGate"),
    (11, r"PoseidonGate\(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>\)<WIDTH=(\d+)>$"),
    (12, r"PoseidonMdsGate\(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>\)<WIDTH=(\d+)>$"),
    (13, r"RandomAccessGate \{ bits: (\d+), num_copies: (\d+), num_extra_constants: (\d+), "
         r"_phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField> \}<D=2>"),
    (14, r"ReducingGate \{ num_coeffs: (\d+)(?:<D=2>)? \}"),
    (15, r"ReducingExtensionGate \{ num_coeffs: (\d+)(?:<D=2>)? \}"),
]


def _gate_words(text: str) -> list:
    """Gate (Gate/Base.hs:27-45) of a Rust Debug string -> [tag, fields...]."""
    import re
    for tag, rx in _GATE_RE:
        m = re.match(rx, text)
        if not m:
            continue
        g = m.groups()
        if tag == 3:
            ws = [int(x) % P for x in g[2].replace(" ", "").split(",") if x]
            return [tag, int(g[0]), int(g[1]), len(ws)] + ws
        if tag in (6, 7):
            hb = [int(x) & 0xFF for x in g[1].replace(" ", "").split(",") if x]
            return [tag, int(g[0]), len(hb)] + hb + ([int(g[2])] if tag == 7 else [])
        return [tag] + [int(x) for x in g]
    name = text.encode()
    return [16, len(name)] + list(name)


def _fri_config_words(fc: dict) -> list:
    rs = fc["reduction_strategy"]
    (k, v), = rs.items()
    tag = {"Fixed": 0, "ConstantArityBits": 1, "MinSize": 2}[k]
    args = [] if v is None else (list(v) if isinstance(v, list) else [v])
    return [fc["rate_bits"], fc["cap_height"], fc["proof_of_work_bits"], tag, len(args)] + args + [fc["num_query_rounds"]]


# scalar fields in word order, by their JSON keys (Types.hs field names without the aeson-dropped
# prefix); tests/test_haskell_shim.py holds bindings/haskell/Plonk/VerifierGPU.hs to the same order
CONFIG_SCALARS = ("num_wires", "num_routed_wires", "num_constants", "use_base_arithmetic_gate", "security_bits",
                  "num_challenges", "zero_knowledge", "randomize_unused_wires", "max_quotient_degree_factor")
COMMON_SCALARS_A = ("quotient_degree_factor", "num_gate_constraints", "num_constants", "num_public_inputs")
COMMON_SCALARS_B = ("num_partial_products", "num_lookup_polys", "num_lookup_selectors")
OPENING_LISTS = ("constants", "plonk_sigmas", "wires", "plonk_zs", "plonk_zs_next", "partial_products", "quotient_polys",
                 "lookup_zs", "lookup_zs_next")


def circuit_words(common_json: Union[str, bytes], vkey_json: Union[str, bytes]) -> np.ndarray:
    """VerifierCircuitData (Types.hs:220-240) as words, from the JSON files it decodes from."""
    import json
    c, vk = json.loads(common_json), json.loads(vkey_json)
    cfg = c["config"]
    w = [WORDS_CIRCUIT_MAGIC] + [int(cfg[k]) for k in CONFIG_SCALARS]
    w += _fri_config_words(cfg["fri_config"])
    fp = c["fri_params"]
    w += _fri_config_words(fp["config"]) + [int(fp["hiding"]), fp["degree_bits"], len(fp["reduction_arity_bits"])]
    w += list(fp["reduction_arity_bits"])
    w += [len(c["gates"])]
    for g in c["gates"]:
        w += _gate_words(g)
    si = c["selectors_info"]
    w += [len(si["selector_indices"])] + list(si["selector_indices"]) + [len(si["groups"])]
    for g in si["groups"]:
        w += [g["start"], g["end"]]
    sv = si.get("selector_vector")
    w += [0] if sv is None else [1, len(sv)] + list(sv)
    w += [c[k] for k in COMMON_SCALARS_A]
    w += [len(c["k_is"])] + [int(x) % P for x in c["k_is"]]
    w += [c[k] for k in COMMON_SCALARS_B] + [len(c["luts"])]
    for t in c["luts"]:
        w += [len(t)]
        for inp, out in t:
            w += [int(inp), int(out)]
    cap = vk["constants_sigmas_cap"]
    w += [len(cap)]
    for d in cap:
        w += [int(x) % P for x in d["elements"]]
    w += [int(x) % P for x in vk["circuit_digest"]["elements"]]
    return np.array([x & _M64 for x in w], dtype=np.uint64)


def proof_words(proof_json: Union[str, bytes]) -> np.ndarray:
    """ProofWithPublicInputs (Types.hs:245-279) as words, from its JSON."""
    import json
    d = json.loads(proof_json)
    pr = d["proof"]
    w = [WORDS_PROOF_MAGIC]

    def cap(c):
        w.append(len(c))
        for dg in c:
            w.extend(int(x) % P for x in dg["elements"])

    def exts(v):
        w.append(len(v))
        for a, b in v:
            w.extend((int(a) % P, int(b) % P))
    cap(pr["wires_cap"])
    cap(pr["plonk_zs_partial_products_cap"])
    cap(pr["quotient_polys_cap"])
    o = pr["openings"]
    for k in OPENING_LISTS:
        exts(o[k])
    fp = pr["opening_proof"]
    w.append(len(fp["commit_phase_merkle_caps"]))
    for c in fp["commit_phase_merkle_caps"]:
        cap(c)
    w.append(len(fp["query_round_proofs"]))
    for q in fp["query_round_proofs"]:
        ep = q["initial_trees_proof"]["evals_proofs"]
        w.append(len(ep))
        for leaf, mp in ep:
            w.append(len(leaf))
            w.extend(int(x) % P for x in leaf)
            cap(mp["siblings"])
        w.append(len(q["steps"]))
        for st in q["steps"]:
            exts(st["evals"])
            cap(st["merkle_proof"]["siblings"])
    exts(fp["final_poly"]["coeffs"])
    w.append(int(fp["pow_witness"]) % P)
    w.append(len(d["public_inputs"]))
    w.extend(int(x) % P for x in d["public_inputs"])
    return np.array([x & _M64 for x in w], dtype=np.uint64)
