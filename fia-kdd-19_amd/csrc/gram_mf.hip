// MF k <= 16 entity Gram caches (the headline's prepare).  Reference: the restricted Hessian
// of total_loss over the related batch (matrix_factorization.py:288-308, 324-351) restated per
// entity, A_e = sum over e's list of g g^T with g = [other-side embedding ; 1].
#include "kern.h"

namespace fia {
namespace {

// raw buffer resource word 3 (gfx9 family)
constexpr int kRsrcWord3 = 0x00020000;

// ------------------------------------------------------------------------------------
// The lists of both sides are cut into sub-batches of 16 ratings (build_gram_stream): a wave
// walks the sub-batches of its range -- whole short lists one after another, or one
// 256-rating slice of a long list -- with one v_mfma_f64_16x16x4_f64 per row-quad (4 per
// sub-batch: a list costs ceil(len / 4) MFMAs, not a padded 64-row batch), and flushes an
// entity's Gram when its last sub-batch is in.  The range's row offsets go to LDS once (stream
// order, quad-transposed: one 16-B LDS read gives a row group its 4 quads' row offsets, and no
// id load sits in front of a gather in the in-order vmcnt queue); the gathered rows run six
// sub-batches ahead of the MFMAs in an 8-slot register ring.  Everything per sub-batch that is
// not a gather or an MFMA was moved out of the loop: the stream holds byte offsets (no
// address arithmetic but the lane's column), a ratings past a list's end is an offset outside
// the table's buffer range (the hardware returns 0: no masking), the per-sub-batch flags are
// bits of three wave masks, a segment's count rides in its last descriptor.  A flush stages
// the packed triangle (+ the bias row: column sums, the count) in LDS and writes it as 16-B
// stores.  fia_prepare_for marks (MARK): the sub-batches of unmarked entities gather past every
// table's range, skip their MFMAs and end no segment.
// Lane map (f64 16x16x4): lane l supplies G[l >> 4][l & 15] of the row-quad as both A (= G^T)
// and B; C register r = C[(l >> 4) + 4 r][l & 15].
// ------------------------------------------------------------------------------------
template <class M, bool MARK>
__global__ __launch_bounds__(64) void k_gram_mf_stream(GramStreamArgs G) {
  static_assert(!M::ncf && M::K <= 16, "MF k <= 16");
  constexpr int K = M::K, Ds = M::Ds, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  static_assert(kGsRing == 8 && kGsMaxSub % kGsRing == 0 && kGsMaxSub + kGsRing <= 64, "ring of 8");
  __shared__ __attribute__((aligned(16))) double stage[kGsMaxSeg][GSP];
  __shared__ uint4 sids[kGsMaxSub * 4];     // [sub-batch][row group] -> the group's 4 row offsets
  const int64_t w = blockIdx.x;
  if (w >= G.n_waves) return;
  const int d0 = G.wave[w], nd = G.wave[w + 1] - d0;     // a multiple of kGsRing, <= kGsMaxSub
  const int lane = threadIdx.x;
  const int col = lane & 15, grp = lane >> 4;
  // the range's descriptors, one per lane, as wave masks: skipped (padding dummies; MARK:
  // unmarked entities), last of a segment, side 1
  const int2 dv = lane < nd ? G.desc[d0 + lane] : int2{1 << 7, 0};
  bool sk = (dv.x >> 7) & 1;
  // (moff picked by a select: a lane-indexed kernel-argument array would go through scratch)
  if constexpr (MARK) sk = sk || !G.mark[((dv.x >> 6) & 1 ? G.moff[1] : G.moff[0]) + (dv.x >> 8)];
  const uint64_t skipm = __ballot(sk), lastm = __ballot((dv.x >> 5) & 1), sidem = __ballot((dv.x >> 6) & 1);
  if (MARK && skipm == ~0ull) return;     // no marked entity in the range
  {
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(G.ids) + (int64_t)d0 * 4;
    uint4 tmp[kGsMaxSub * 4 / 64];
#pragma unroll
    for (int r = 0; r < kGsMaxSub * 4 / 64; ++r) {
      const int i = r * 64 + lane;
      tmp[r] = src[i < nd * 4 ? i : 0];
    }
#pragma unroll
    for (int r = 0; r < kGsMaxSub * 4 / 64; ++r) sids[r * 64 + lane] = tmp[r];
    wave_lds_sync();
  }
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.emb_other[0]), 0, G.bytes_other[0], kRsrcWord3);
  const __amdgpu_buffer_rsrc_t rs1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.emb_other[1]), 0, G.bytes_other[1], kRsrcWord3);
  // the lane's column bytes; columns >= k land past every table (kGsNoRow-sized offsets + this
  // stay outside the range too)
  const uint32_t cb = col < K ? (uint32_t)col * 4u : 0x80000000u;
  // rows of sub-batch t: quad q, row group grp -> rating 4 q + grp of the sub-batch
  auto rows = [&](int t, float (&v)[4]) {
    const __amdgpu_buffer_rsrc_t rs = (sidem >> t) & 1 ? rs1 : rs0;
    // a look-ahead gather past the range's end (t >= nd) and, MARK, a skipped sub-batch get the
    // top offset bit: outside every table, the hardware returns 0 without touching memory.  (A
    // third, empty resource picked here instead went to scratch and a readfirstlane loop per
    // gather.)
    const uint32_t sb = t >= nd || (MARK && ((skipm >> t) & 1)) ? 0x80000000u : 0u;
    const uint4 o4 = sids[(t < nd ? t : 0) * 4 + grp];
    const uint32_t oq[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t off = (oq[q] + cb) | sb;
      v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0));
    }
  };
  // two accumulators (even / odd row-quads): consecutive MFMAs are independent
  d4_t acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  double sum = 0.0;
  int nseg = 0;                            // segments flushed so far (their Grams in stage[])
  auto step = [&](int t, const float (&vin)[4]) {
    if ((skipm >> t) & 1) return;
    // the slot's values pass an empty asm here: the converts (and the wait for the gathers)
    // stay at this sub-batch instead of being hoisted to the loop head with the others
    float v[4] = {vin[0], vin[1], vin[2], vin[3]};
    asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
    double g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) g[q] = (double)v[q];
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(g[0], g[0], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(g[1], g[1], acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(g[2], g[2], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(g[3], g[3], acc1, 0, 0, 0);
    sum += (g[0] + g[1]) + (g[2] + g[3]);
    if (!((lastm >> t) & 1)) return;
    // the entity's (or the slice's) Gram -- packed lower triangle, bias row, count -- staged in
    // LDS; the global stores wait for the end of the range (a store in the middle of the ring
    // stalled the wave behind the gathers in flight: ~60 % of this kernel's time)
    const uint32_t out = (uint32_t)__builtin_amdgcn_readlane(dv.y, t);
    double* __restrict__ st = stage[nseg];
    double cs = sum;
    cs += __shfl_xor(cs, 16);
    cs += __shfl_xor(cs, 32);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = grp + 4 * rr;
      if (row < K && col <= row) st[tri(row, col)] = acc0[rr] + acc1[rr];
    }
    if (grp == 0 && col < K) st[tri(K, col)] = cs;
    if (lane == 0) st[tri(K, K)] = (double)(out >> 23);
    if (GSP > GS && lane == 1) st[GSP - 1] = 0.0;
    ++nseg;
    acc0 = acc1 = d4_t{0.0, 0.0, 0.0, 0.0};
    sum = 0.0;
  };
  // kGsRing-slot register ring, gathers kGsRing - 2 sub-batches ahead of the MFMAs (slots
  // named statically: one ring turn per loop trip; past the range's end every offset carries
  // the top bit, see rows())
  constexpr int AH = kGsRing - 2;
  float r[kGsRing][4];
#pragma unroll
  for (int j = 0; j < AH; ++j) rows(j, r[j]);
  for (int t = 0; t < nd; t += kGsRing) {
#pragma unroll
    for (int j = 0; j < kGsRing; ++j) {
      rows(t + j + AH, r[(j + AH) % kGsRing]);
      step(t + j, r[j]);
    }
  }
  // the range's Grams, in segment order: segment k ends at the k-th descriptor that is the last
  // of a segment and not skipped
  wave_lds_sync();
  uint64_t ends = lastm & ~skipm;
  for (int k = 0; k < nseg; ++k) {
    const int t = (int)__builtin_ctzll(ends);
    ends &= ends - 1;
    const int meta = __builtin_amdgcn_readlane(dv.x, t);
    const uint32_t out = (uint32_t)__builtin_amdgcn_readlane(dv.y, t);
    const int sd = (meta >> 6) & 1, e = meta >> 8, slot = (int)(out & 0x7fffffu) - 1;
    double* __restrict__ o = slot < 0 ? G.gram[sd] + (int64_t)e * GSP : G.part[sd] + (int64_t)slot * GSP;
#pragma unroll
    for (int b = 0; b < GSP; b += 128)
      if (b + 2 * lane < GSP)
        *reinterpret_cast<double2*>(o + b + 2 * lane) = *reinterpret_cast<const double2*>(&stage[k][b + 2 * lane]);
  }
}

}  // namespace

hipError_t launch_gram_mf_stream(int k, const GramStreamArgs& G, hipStream_t s) {
  if (G.n_waves <= 0) return hipSuccess;
  const dim3 grid((unsigned)G.n_waves), blk(64);
  if (k == 16) {
    if (G.mark) hipLaunchKernelGGL((k_gram_mf_stream<MFm<16>, true>), grid, blk, 0, s, G);
    else hipLaunchKernelGGL((k_gram_mf_stream<MFm<16>, false>), grid, blk, 0, s, G);
  } else if (k == 8) {
    if (G.mark) hipLaunchKernelGGL((k_gram_mf_stream<MFm<8>, true>), grid, blk, 0, s, G);
    else hipLaunchKernelGGL((k_gram_mf_stream<MFm<8>, false>), grid, blk, 0, s, G);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace fia
