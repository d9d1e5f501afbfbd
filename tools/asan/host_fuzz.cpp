// host_fuzz.cpp — AddressSanitizer / UBSan run of libp2v's host readers (circuit.cpp, json.hpp):
// the JSON circuit and proof readers, the template-guided packer, the word and byte readers, fed
// seeded mutations (truncations, byte flips, inserted bytes) of real inputs.  Host code only (the
// GPU cannot run sanitizers on this pool).  Build and run: tools/asan/run.sh
#include "../../plonky2-verifier_amd/csrc/circuit.hpp"
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

using namespace p2v;

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss; ss << f.rdbuf();
  return ss.str();
}

template <class F>
static int guarded(F&& f) {
  try { f(); return 0; } catch (const ShapeError&) { return 1; } catch (const ParseError&) { return 2; }
  catch (const CircuitError&) { return 3; } catch (const std::exception&) { return 4; }
}

static std::string mutate(const std::string& s, std::mt19937_64& rng) {
  std::string d = s;
  switch (rng() % 3) {
    case 0: d.resize(rng() % (d.size() + 1)); break;
    case 1: for (int k = 1 + rng() % 5; k-- > 0 && !d.empty();) d[rng() % d.size()] = (char)(rng() & 0xff); break;
    default: { size_t i = d.empty() ? 0 : rng() % d.size(); d.insert(i, std::string(1 + rng() % 40, (char)(rng() & 0xff))); }
  }
  return d;
}

int main(int argc, char** argv) {
  if (argc < 7) { fprintf(stderr, "usage: %s common.json vkey.json proof.json proof.bin circuit.words proof.words [iters]\n", argv[0]); return 2; }
  const std::string common = slurp(argv[1]), vkey = slurp(argv[2]), proof = slurp(argv[3]), bin = slurp(argv[4]);
  const std::string cw = slurp(argv[5]), pw = slurp(argv[6]);
  const int iters = argc > 7 ? atoi(argv[7]) : 2000;
  Circuit C = parse_circuit(parse_json(common.data(), common.size()), parse_json(vkey.data(), vkey.size()));
  std::vector<uint64_t> ref(C.L.words), out(C.L.words);
  pack_proof(C, parse_json(proof.data(), proof.size()), ref.data());
  pack_proof_bytes(C, (const uint8_t*)bin.data(), bin.size(), out.data());
  if (out != ref) { fprintf(stderr, "bytes path != JSON path\n"); return 1; }
  Circuit Cw = parse_circuit_words((const uint64_t*)cw.data(), cw.size() / 8);
  pack_proof_words(Cw, (const uint64_t*)pw.data(), pw.size() / 8, out.data());
  if (out != ref) { fprintf(stderr, "words path != JSON path\n"); return 1; }
  ProofTemplate T;
  if (!T.build(C, proof.data(), proof.size(), out.data()) || out != ref) { fprintf(stderr, "template build\n"); return 1; }
  // huge Int fields must be rejected before the reduction strategy is expanded (no
  // unbounded allocation, no truncating casts).  Word layout with ConstantArityBits: [9] config
  // scalars, FriConfig at 10 (tag 13, 2 args at 15 16), FriParams' FriConfig at 18, degree_bits 27.
  if (cw.size() / 8 < 28 || ((const uint64_t*)cw.data())[13] != 1 || ((const uint64_t*)cw.data())[14] != 2) {
    fprintf(stderr, "unexpected circuit word layout\n"); return 1;
  }
  struct Crafted { int idx[3]; uint64_t val[3]; int want; const char* what; };
  const Crafted crafted[] = {
    {{27, 15, 16}, {0x7FFFFFFFull, 1, (uint64_t)-(int64_t)1000000000}, 3, "degree_bits 2^31-1, arity 1, final_poly_bits -1e9"},
    {{27, -1, -1}, {1ull << 40, 0, 0}, 2, "degree_bits 2^40 (past int)"},
    {{1, -1, -1}, {(uint64_t)-(int64_t)(1ll << 35), 0, 0}, 2, "num_wires -2^35"},
    {{16, -1, -1}, {(uint64_t)-(int64_t)(1ll << 33), 0, 0}, 3, "final_poly_bits -2^33"},
  };
  for (const auto& k : crafted) {
    std::string x = cw;
    for (int j = 0; j < 3; j++) if (k.idx[j] >= 0) ((uint64_t*)&x[0])[k.idx[j]] = k.val[j];
    const int got = guarded([&] { Circuit X = parse_circuit_words((const uint64_t*)x.data(), x.size() / 8); });
    if (got != k.want) { fprintf(stderr, "crafted words (%s): class %d, expected %d\n", k.what, got, k.want); return 1; }
  }
  {
    std::string j = common;
    const size_t at = j.find("\"degree_bits\":");
    if (at == std::string::npos) { fprintf(stderr, "no degree_bits\n"); return 1; }
    j.insert(at + 14, "2147483647000");   // a number past int: rejected, not truncated
    const int got = guarded([&] { Circuit X = parse_circuit(parse_json(j.data(), j.size()), parse_json(vkey.data(), vkey.size())); });
    if (got != 2) { fprintf(stderr, "crafted JSON degree_bits: class %d, expected 2 (parse)\n", got); return 1; }
  }
  std::mt19937_64 rng(12345);
  int counts[5] = {0, 0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
    const std::string pj = mutate(proof, rng), pb = mutate(bin, rng), cj = mutate(common, rng);
    std::string pwm = mutate(pw, rng); pwm.resize(pwm.size() / 8 * 8);
    std::string cwm = mutate(cw, rng); cwm.resize(cwm.size() / 8 * 8);
    counts[guarded([&] { pack_proof(C, parse_json(pj.data(), pj.size()), out.data()); })]++;
    counts[guarded([&] { if (!T.pack(pj.data(), pj.size(), out.data())) throw ParseError("off template"); })]++;
    counts[guarded([&] { pack_proof_bytes(C, (const uint8_t*)pb.data(), pb.size(), out.data()); })]++;
    counts[guarded([&] { pack_proof_words(C, (const uint64_t*)pwm.data(), pwm.size() / 8, out.data()); })]++;
    counts[guarded([&] { Circuit X = parse_circuit(parse_json(cj.data(), cj.size()), parse_json(vkey.data(), vkey.size())); })]++;
    counts[guarded([&] { Circuit X = parse_circuit_words((const uint64_t*)cwm.data(), cwm.size() / 8); })]++;
  }
  printf("{\"iters\": %d, \"ok\": %d, \"shape\": %d, \"parse\": %d, \"circuit\": %d, \"other\": %d}\n", iters, counts[0], counts[1],
         counts[2], counts[3], counts[4]);
  return 0;
}
