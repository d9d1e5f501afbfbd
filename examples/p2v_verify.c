/*
 * p2v_verify — verify Plonky2 proofs from the reference's JSON files through the C ABI only
 * (no Python): what a non-Python host (the Haskell shim of INTEGRATION.md, a C++ service)
 * does with libp2v.
 *
 *   p2v_verify [--pack-only] [--devices N] [--dump FILE] common.json vkey.json proof.json [proof.json ...]
 *   p2v_verify --words [...] circuit.words proof.words [proof.words ...]
 *   p2v_verify --bytes [...] common.json vkey.json proof.bin [proof.bin ...]
 *
 * Prints one line per proof, "<file> <status>": 1 True, 0 False, < 0 the class of `error`
 * the reference would raise (include/p2v.h).  With --pack-only the proofs are decoded and
 * packed (host only, no GPU) and each line carries the packed word count instead.
 * --devices N shards the batch over devices 0..N-1 (p2v_verify_batch_devices).
 * --words: the inputs are the word-encoded Types.hs values (little-endian u64 files, the
 * layout of include/p2v.h that a typed host such as the Haskell shim writes) instead of JSON:
 * p2v_circuit_from_words + p2v_pack_proof_words.  --bytes: the proofs are plonky2's binary
 * serialization (p2v_pack_proof_bytes).  --ext FLAGS: opt-in plonky2 conventions (P2V_EXT_*,
 * p2v_circuit_from_*_ex).  --dump FILE writes the packed words.
 * Exit: 0 done, 2 usage / IO, 3 circuit rejected, 4 a proof did not decode, 5 device error.
 *
 * Build: gcc -O2 -I include examples/p2v_verify.c -L plonky2-verifier_amd -lp2v \
 *            -Wl,-rpath,$PWD/plonky2-verifier_amd -o p2v_verify
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "p2v.h"

static char* read_file(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* buf = (char*)malloc((size_t)n + 1);
  if (buf && fread(buf, 1, (size_t)n, f) != (size_t)n) { free(buf); buf = NULL; }
  fclose(f);
  if (buf) { buf[n] = 0; *len = (size_t)n; }
  return buf;
}

int main(int argc, char** argv) {
  int pack_only = 0, ndev = 1, a = 1, wordsin = 0, bytesin = 0;
  uint32_t ext = 0;
  const char* dump = NULL;
  for (; a < argc && argv[a][0] == '-' && argv[a][1] == '-'; a++) {
    if (!strcmp(argv[a], "--pack-only")) pack_only = 1;
    else if (!strcmp(argv[a], "--words")) wordsin = 1;
    else if (!strcmp(argv[a], "--bytes")) bytesin = 1;
    else if (!strcmp(argv[a], "--ext") && a + 1 < argc) ext = (uint32_t)strtoul(argv[++a], NULL, 0);
    else if (!strcmp(argv[a], "--devices") && a + 1 < argc) ndev = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--dump") && a + 1 < argc) dump = argv[++a];
    else { fprintf(stderr, "unknown option %s\n", argv[a]); return 2; }
  }
  const int nhdr = wordsin ? 1 : 2;   /* circuit.words | common.json vkey.json */
  if (argc - a < nhdr + 1 || ndev < 1 || (wordsin && bytesin)) {
    fprintf(stderr, "usage: %s [--pack-only] [--devices N] [--dump FILE] [--ext FLAGS] common.json vkey.json proof.json...\n"
                    "       %s --words [...] circuit.words proof.words...\n"
                    "       %s --bytes [...] common.json vkey.json proof.bin...\n", argv[0], argv[0], argv[0]);
    return 2;
  }
  size_t clen = 0, vlen = 0;
  char* common = read_file(argv[a], &clen);
  char* vkey = wordsin ? NULL : read_file(argv[a + 1], &vlen);
  if (!common || (!wordsin && !vkey)) { fprintf(stderr, "cannot read the circuit files\n"); return 2; }
  p2v_circuit* circ = NULL;
  int crc = wordsin ? p2v_circuit_from_words_ex((const uint64_t*)common, clen / 8, ext, &circ)
                    : p2v_circuit_from_json_ex(common, clen, vkey, vlen, ext, &circ);
  if (crc != P2V_OK) {
    fprintf(stderr, "circuit: %s\n", p2v_last_error_message());
    return 3;
  }
  p2v_circuit_info info;
  p2v_circuit_get_info(circ, &info);
  const int n = argc - a - nhdr;
  const char** texts = (const char**)calloc((size_t)n, sizeof(char*));
  size_t* lens = (size_t*)calloc((size_t)n, sizeof(size_t));
  for (int i = 0; i < n; i++) {
    texts[i] = read_file(argv[a + nhdr + i], &lens[i]);
    if (!texts[i]) { fprintf(stderr, "cannot read %s\n", argv[a + nhdr + i]); return 2; }
  }
  uint64_t* words = (uint64_t*)malloc((size_t)n * (size_t)info.proof_words * sizeof(uint64_t));
  int32_t* codes = (int32_t*)malloc((size_t)n * sizeof(int32_t));
  if (wordsin || bytesin) {
    for (int i = 0; i < n; i++) {
      uint64_t* dst = words + (size_t)i * (size_t)info.proof_words;
      const int rc = wordsin ? p2v_pack_proof_words(circ, (const uint64_t*)texts[i], lens[i] / 8, dst)
                             : p2v_pack_proof_bytes(circ, (const uint8_t*)texts[i], lens[i], dst);
      if (rc != P2V_OK) {
        fprintf(stderr, "%s: %s\n", argv[a + nhdr + i], p2v_last_error_message());
        return 4;
      }
    }
  } else if (p2v_pack_proofs_json(circ, texts, lens, (size_t)n, words, codes, 0) != 0) {
    for (int i = 0; i < n; i++)
      if (codes[i] != P2V_OK) fprintf(stderr, "%s: decode error %d\n", argv[a + nhdr + i], codes[i]);
    fprintf(stderr, "%s\n", p2v_last_error_message());
    return 4;
  }
  if (dump) {
    FILE* f = fopen(dump, "wb");
    if (!f || fwrite(words, 8, (size_t)n * (size_t)info.proof_words, f) != (size_t)n * (size_t)info.proof_words) { fprintf(stderr, "cannot write %s\n", dump); return 2; }
    fclose(f);
  }
  int rc = 0;
  if (pack_only) {
    for (int i = 0; i < n; i++) printf("%s %lld\n", argv[a + nhdr + i], (long long)info.proof_words);
  } else {
    int8_t* res = (int8_t*)malloc((size_t)n);
    int* devs = (int*)malloc((size_t)ndev * sizeof(int));
    for (int d = 0; d < ndev; d++) devs[d] = d;
    int e = ndev > 1 ? p2v_verify_batch_devices(circ, words, (size_t)n, res, devs, ndev, 0)
                     : p2v_verify_batch(circ, words, (size_t)n, res, 0);
    if (e != P2V_OK) {
      fprintf(stderr, "verify: %s\n", p2v_last_error_message());
      rc = 5;
    } else {
      for (int i = 0; i < n; i++) printf("%s %d\n", argv[a + nhdr + i], (int)res[i]);
    }
    free(res);
    free(devs);
  }
  for (int i = 0; i < n; i++) free((void*)texts[i]);
  free(texts); free(lens); free(words); free(codes); free(common); free(vkey);
  p2v_circuit_free(circ);
  return rc;
}
