// merkle.hip — the top levels of the Merkle paths, each distinct node compressed once per proof
// (Hash/Merkle.hs:27-42, verifyMerkleProofToCap).
//
// A proof's 28 query paths of one tree meet near the cap: at the absolute level A (A halvings
// from the initial trees' leaves) query q sits at node idx_q >> A, the same for every tree (a
// step tree's leaf index is idx >> sh and its paths end at A = lde_bits - cap_height = Ltop, like
// the initial trees').  With 2^(Ltop - A) nodes at level A, 28 queries occupy on average 13.4
// of the 16 nodes below a height-4 cap, 18.8 of 32, 22.9 of 64, 25.2 of 128, 26.6 of 256: of the
// 5 x 28 = 140 compressions of a path's top five levels, 107 are distinct.  Per proof that is
// ~194 of the 1 512 Merkle compressions (6 trees), 7 % of all 2 775 permutations.
//
// k_merkle compresses every path up to Ltop - K_t (K_t = min(mt_K, depth_t), DevCircuit::mt_k)
// and leaves that node in leafdig.  Then, per proof:
//   k_mtask   the query q is the group representative at level A when no q' < q shares its node
//             (rep_A(q) = min{q' : idx_q' >> A == idx_q >> A}); representation is monotone in A,
//             so q compresses a run of n_q consecutive top levels.  Tasks (p, q) are bucketed by
//             (K_t, n_q) so that a wave's 64 tasks run the same number of compressions.
//   k_mtop    each task's chain of n_q compressions from leafdig[q][t], every level's value kept
//             in mt_val (gathers: a wave's lanes are arbitrary (proof, query) pairs).
//   k_mcheck  equality, not hashing (then k_mcap writes the unflagged trees' results): a query q that is not the representative h of its level-A
//             group has the same compression input as h exactly when (same child node) its
//             sibling equals h's (and, at the first top level, its own bottom value equals h's) or
//             (sibling children) its child value equals h's sibling and its sibling equals h's
//             child value.  Then its path value at A is h's, by induction up to the cap, and its
//             Merkle check is h's root against cap[idx_q >> Ltop] -- the reference's per-query
//             result, with no assumption about the hash.  A (proof, tree) with any inequality is
//             listed for k_mfix.
//   k_mfix    recomputes the listed trees' top levels per query, without sharing (the corrupted
//             proofs' trees in practice), so every status equals the per-path verification.
#include "devcommon.h"

using namespace p2d;

namespace {

// idx of query q of proof p, shifted into tree t's leaf index space, and t's path geometry
__device__ __forceinline__ int tree_shift(const DevCircuit& c, int t) {
  if (t < 4) return 0;
  int sh = 0;
  for (int j = 0; j <= t - 4; j++) sh += c.arity[j];
  return sh;
}
__device__ __forceinline__ int tree_depth(const DevCircuit& c, int t) { return t < 4 ? c.depth0 : c.step_depth[t - 4]; }
__device__ __forceinline__ int64_t tree_path(const DevCircuit& c, int t, int q) {
  return c.q0 + (int64_t)q * c.qstride + (t < 4 ? c.path[t] : c.step_path[t - 4]);
}
// cap_roots of tree t, entry ci, word i (Merkle.hs:44-47)
__device__ __forceinline__ uint64_t cap_root(const DevCircuit& c, int t, uint32_t ci, int i, int p) {
  if (t == 0) return c.cs_cap[ci * 4 + i];
  if (t == 1) return ld(c, c.wcap + ci * 4 + i, p);
  if (t == 2) return ld(c, c.zcap + ci * 4 + i, p);
  if (t == 3) return ld(c, c.qcap + ci * 4 + i, p);
  return ld(c, c.ccaps + (int64_t)(t - 4) * 4 * c.cap_len + ci * 4 + i, p);
}
// compress(cur, sib) if the node index is even, compress(sib, cur) if odd (Merkle.hs:33-37)
__device__ __forceinline__ void compress_up(uint64_t cur[4], const uint64_t sib[4], bool odd) {
  uint64_t st[12];
#pragma unroll
  for (int i = 0; i < 4; i++) { st[i] = odd ? sib[i] : cur[i]; st[4 + i] = odd ? cur[i] : sib[i]; st[8 + i] = 0; }
  p2::permute_dev(st, true, 1);
#pragma unroll
  for (int i = 0; i < 4; i++) cur[i] = st[i];
}
__device__ __forceinline__ uint32_t qidx(const DevCircuit& c, int q, int p) { return (uint32_t)chal(c, CH_QIDX(c) + q, p); }
// mt_val slot of absolute level A, tree-independent: A = Ltop - mt_K + 1 + slot
__device__ __forceinline__ uint64_t* mt_slot(const DevCircuit& c, int A, int q, int t, int p) {
  const int s = A - (c.mt_L - c.mt_K + 1);
  return c.mt_val + ((((int64_t)s * c.Q + q) * c.T + t) * 4) * c.B + p;
}
// the group representative of q at absolute level A (lowest query index on q's node)
__device__ __forceinline__ int rep_at(const DevCircuit& c, int q, uint32_t iq, int A, int p) {
  int h = q;
  for (int k = q - 1; k >= 0; k--) if (((qidx(c, k, p) ^ iq) >> A) == 0) h = k;
  return h;
}
// bucket (K class, n) of the task lists
__device__ __forceinline__ int64_t bucket(const DevCircuit& c, int kc, int n) { return (int64_t)kc * (c.mt_K + 1) + n; }

}  // namespace

// one lane per (query, proof), a wave = one query of 64 proofs: bucket the (proof, query) task by
// its run length; one atomic per wave and bucket, tasks appended in proof order (so that a
// chunk's lanes mostly read one 512-B row of the tiled batch per word)
extern "C" __global__ void __launch_bounds__(256) k_mtask(DevCircuit c) {
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NPB = c.B >> 6;
  if (unit >= c.Q * NPB) return;
  const int q = unit / NPB, p = (unit % NPB) * 64 + lane;
  const bool live = p < c.n;
  // highest level at which q is still alone among q' < q: the merge level of (q', q) is the
  // bit length of idx_q' ^ idx_q
  const uint32_t iq = qidx(c, q, p);
  int m = 64;
  for (int k = 0; k < q; k++) {
    const uint32_t x = qidx(c, k, p) ^ iq;
    const int mm = x ? 32 - __clz((int)x) : 0;
    m = mm < m ? mm : m;
  }
  const int r = m - 1;   // q represents its node at every level A <= r
  for (int kc = 0; kc < c.mt_ncls; kc++) {
    const int K = c.mt_kval[kc];
    int n = r - (c.mt_L - K);
    n = n < 0 ? 0 : (n > K ? K : n);
    if (!live) n = 0;
    for (int nn = 1; nn <= K; nn++) {
      const uint64_t mask = __ballot(n == nn);
      if (!mask) continue;
      const int leader = __ffsll((unsigned long long)mask) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(c.mt_cnt + bucket(c, kc, nn), __popcll(mask));
      base = __shfl(base, leader);
      if (n == nn) {
        const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
        c.mt_task[bucket(c, kc, nn) * (int64_t)c.B * c.Q + pos] = ((uint32_t)p << 8) | (uint32_t)q;
      }
    }
  }
}

// chains: one wave per 64-task chunk of one (n, tree) bucket, longest chains first; the grid is
// the host's bound on the chunk count (per tree n_proofs Q / 64 + K_t), waves past the actual
// count exit at once
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) k_mtop(DevCircuit c) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  // locate (n, t, offset): n descending, trees in order (wave-uniform)
  int tsel = -1, nsel = 0, off = 0, cnt = 0, kc = 0;
  {
    int acc = 0;
    for (int n = c.mt_K; n >= 1 && tsel < 0; n--)
      for (int t = 0; t < c.T && tsel < 0; t++) {
        const int K = c.mt_k[t];
        if (K < n) continue;
        const int k = c.mt_kcls[K];
        const int ct = c.mt_cnt[bucket(c, k, n)];
        const int ch = (ct + 63) >> 6;
        if (chunk < acc + ch) { tsel = t; nsel = n; off = chunk - acc; cnt = ct; kc = k; }
        acc += ch;
      }
  }
  if (tsel < 0) return;
  // a partial last chunk: its idle lanes repeat the chunk's first task and store nothing
  const int i = off * 64 + lane;
  const bool act = i < cnt;
  const uint32_t task = c.mt_task[bucket(c, kc, nsel) * (int64_t)c.B * c.Q + (act ? i : off * 64)];
  const int p = (int)(task >> 8), q = (int)(task & 255u);
  const int t = tsel;
  const int K = c.mt_k[t], d = tree_depth(c, t), sh = tree_shift(c, t);
  const int l0 = d - K;
  uint32_t idx = qidx(c, q, p) >> (sh + l0);
  const int64_t poff = tree_path(c, t, q);
  const uint64_t* src = c.leafdig + ((int64_t)(q * c.T + t) * 4) * c.B + p;
  uint64_t cur[4];
#pragma unroll
  for (int w = 0; w < 4; w++) cur[w] = src[(int64_t)w * c.B];
  for (int j = 0; j < nsel; j++) {
    const int l = l0 + j;
    uint64_t sib[4];
#pragma unroll
    for (int w = 0; w < 4; w++) sib[w] = ld(c, poff + 4 * l + w, p);
    compress_up(cur, sib, idx & 1u);
    idx >>= 1;
    if (act) {
      uint64_t* dst = mt_slot(c, sh + l + 1, q, t, p);
#pragma unroll
      for (int w = 0; w < 4; w++) dst[(int64_t)w * c.B] = cur[w];
    }
  }
}

// the top trees' units (tree, query, 64 proofs), a wave each: unit -> (t, q, p); false past the batch
__device__ __forceinline__ bool top_unit(const DevCircuit& c, int& t, int& q, int& p) {
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NPB = c.B >> 6;
  int u = unit / (c.Q * NPB);
  q = (unit / NPB) % c.Q;
  p = (unit % NPB) * 64 + (threadIdx.x & 63);
  for (t = 0; t < c.T; t++) if (c.mt_k[t] > 0 && u-- == 0) break;
  return t < c.T && p < c.n;
}

// one lane per (tree, query, proof): the equality checks of q's compressions in the shared levels;
// a (proof, tree) with any inequality is flagged and listed (once) for k_mfix
extern "C" __global__ void __launch_bounds__(256) k_mcheck(DevCircuit c) {
  int t, q, p;
  if (!top_unit(c, t, q, p)) return;
  const int Lt = c.mt_L;
  const int K = c.mt_k[t], d = tree_depth(c, t);
  const uint32_t iq = qidx(c, q, p);
  const int64_t pq = tree_path(c, t, q);
  bool bad = false;
  for (int j = 0; j < K; j++) {
    const int A = Lt - K + 1 + j;       // output level of this compression
    const int h = rep_at(c, q, iq, A, p);
    if (h == q) continue;
    const int l = d - K + j;            // compression index in tree t's paths
    const int64_t ph = tree_path(c, t, h);
    const uint32_t ih = qidx(c, h, p);
    const bool same = ((ih ^ iq) >> (A - 1)) == 0;
    const int rq = j == 0 ? q : rep_at(c, q, iq, A - 1, p);
    for (int w = 0; w < 4; w++) {
      const uint64_t sq = ld(c, pq + 4 * l + w, p), shh = ld(c, ph + 4 * l + w, p);
      uint64_t vq, vh;   // path values entering the compression
      if (j == 0) {
        vq = c.leafdig[((int64_t)(q * c.T + t) * 4 + w) * c.B + p];
        vh = c.leafdig[((int64_t)(h * c.T + t) * 4 + w) * c.B + p];
      } else {
        vq = mt_slot(c, A - 1, rq, t, p)[(int64_t)w * c.B];
        vh = mt_slot(c, A - 1, h, t, p)[(int64_t)w * c.B];
      }
      if (same) bad = bad || sq != shh || (j == 0 && vq != vh);
      else bad = bad || vq != shh || sq != vh;
    }
  }
  if (bad && atomicOr(c.mt_flag + (int64_t)t * c.B + p, 1) == 0) {
    const int slot = atomicAdd(c.mt_cnt + c.mt_nbuckets, 1);
    c.mt_fix[slot] = ((uint32_t)p << 8) | (uint32_t)t;
  }
}

// one lane per (tree, query, proof) of an unflagged (proof, tree): q's Merkle result is its
// top-level representative's root against cap[idx_q >> Ltop]
extern "C" __global__ void __launch_bounds__(256) k_mcap(DevCircuit c) {
  int t, q, p;
  if (!top_unit(c, t, q, p)) return;
  if (c.mt_flag[(int64_t)t * c.B + p]) return;   // k_mfix writes this tree's results
  const int Lt = c.mt_L;
  const uint32_t iq = qidx(c, q, p);
  const uint32_t ci = iq >> Lt;
  const int h = rep_at(c, q, iq, Lt, p);
  const uint64_t* root = mt_slot(c, Lt, h, t, p);
  bool ok = ci < (uint32_t)c.cap_len;
  const uint32_t cc = ok ? ci : 0;
  for (int w = 0; w < 4; w++) ok = ok && root[(int64_t)w * c.B] == cap_root(c, t, cc, w, p);
  c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = ok ? 1 : 0;
}

// listed (proof, tree) pairs: every query's top levels from its own bottom value and siblings
extern "C" __global__ void __launch_bounds__(256) k_mfix(DevCircuit c) {
  const int nfix = c.mt_cnt[c.mt_nbuckets];
  const int total = nfix * c.Q;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int e = i / c.Q, q = i % c.Q;
    const uint32_t f = c.mt_fix[e];
    const int p = (int)(f >> 8), t = (int)(f & 255u);
    const int K = c.mt_k[t], d = tree_depth(c, t), sh = tree_shift(c, t);
    const int l0 = d - K;
    uint32_t idx = qidx(c, q, p) >> (sh + l0);
    const int64_t poff = tree_path(c, t, q);
    const uint64_t* src = c.leafdig + ((int64_t)(q * c.T + t) * 4) * c.B + p;
    uint64_t cur[4];
    for (int w = 0; w < 4; w++) cur[w] = src[(int64_t)w * c.B];
    for (int l = l0; l < d; l++) {
      uint64_t sib[4];
      for (int w = 0; w < 4; w++) sib[w] = ld(c, poff + 4 * l + w, p);
      compress_up(cur, sib, idx & 1u);
      idx >>= 1;
    }
    bool ok = idx < (uint32_t)c.cap_len;
    const uint32_t cc = ok ? idx : 0;
    for (int w = 0; w < 4; w++) ok = ok && cur[w] == cap_root(c, t, cc, w, p);
    c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = ok ? 1 : 0;
  }
}
