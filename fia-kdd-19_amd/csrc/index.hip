// Rating index (CSR by user, CSC by item), related-set counting and the
// per-batch chunk list.
//
// Replaces the reference's per-query O(N) scans
//   u_indices = np.where(train.x[:, 0] == test_u)   (matrix_factorization.py:320)
//   i_indices = np.where(train.x[:, 1] == test_i)   (matrix_factorization.py:321)
// with a one-time stable radix sort: inside every list train rows stay in
// ascending order, so rel(u,i) = R_u ++ C_i is the reference's concatenation
// bit for bit (mf:322).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "common.h"

namespace fia {
namespace {

__global__ void k_check_ids(const int32_t* __restrict__ user, const int32_t* __restrict__ item, int64_t N,
                            int64_t U, int64_t I, int32_t* __restrict__ flag) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int bad = 0;
  for (; j < N; j += stride) {
    int32_t u = user[j], i = item[j];
    bad |= (u < 0 || u >= U || i < 0 || i >= I);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void k_gather_side(const int32_t* __restrict__ rows, const int32_t* __restrict__ other_src,
                              const float* __restrict__ rating_src, int64_t N, int32_t* __restrict__ other,
                              float* __restrict__ rating) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; j < N; j += stride) {
    int32_t r = rows[j];
    other[j] = other_src[r];
    rating[j] = rating_src[r];
  }
}

// pair set insert: one slot per distinct (u, i), counting duplicate train rows
__global__ void k_pair_insert(const int32_t* __restrict__ user, const int32_t* __restrict__ item,
                              const float* __restrict__ rating, int64_t N, int64_t I, unsigned long long* key,
                              int32_t* cnt, double* sum, unsigned long long mask) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; j < N; j += stride) {
    const unsigned long long k = (unsigned long long)user[j] * (unsigned long long)I + (unsigned long long)item[j];
    unsigned long long h = pair_hash(k) & mask;
    for (unsigned long long probe = 0; probe <= mask; ++probe) {
      unsigned long long prev = atomicCAS(&key[h], kEmptyKey, k);
      if (prev == kEmptyKey || prev == k) {
        atomicAdd(&cnt[h], 1);
        atomicAdd(&sum[h], (double)rating[j]);
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

// ptr[e] = lower_bound(sorted_keys, e), e in [0, n_entity]
__global__ void k_list_ptr(const int32_t* __restrict__ keys, int64_t N, int64_t n_entity, int64_t* __restrict__ ptr) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e > n_entity) return;
  int64_t lo = 0, hi = N;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < e) lo = mid + 1; else hi = mid;
  }
  ptr[e] = lo;
}

__device__ inline void query_sides(const int32_t* qu, const int32_t* qi, int64_t q, const int64_t* uptr,
                                   const int64_t* iptr, int64_t U, int64_t I, int64_t& ub, int64_t& du, int64_t& ib,
                                   int64_t& di) {
  const int32_t u = qu[q], i = qi[q];
  ub = du = ib = di = 0;
  if (u >= 0 && u < U && i >= 0 && i < I) {
    ub = uptr[u];
    du = uptr[u + 1] - ub;
    ib = iptr[i];
    di = iptr[i + 1] - ib;
  }
}

// ---- single-pass per-query scans (decoupled look-back) ----
// One launch replaces count kernel + two-kernel library scan (+ descriptor fill): tiles of
// kScanTile queries take a dynamic tile number, publish their aggregate, look back over
// the earlier tiles' words {flag (2 bits), value (62 bits)} and write the exclusive
// prefix of every query (+ the total at [Q]).  The last tile to finish clears the tile
// words and counters, so no memset precedes the next launch.
//   MODE 0: n_q = |R_u| + |C_i| -> offsets (fia_count_related); bad ids flag[1]
//   MODE 1: chunks_q = ceil(|R_u|/kChunk) + ceil(|C_i|/kChunk) -> coff, + chunk descriptors
// (ml-1m-ex, both scans per step, same-box A/B: tiles of 64 / 128 / 256 / 512 / 1024 queries
// 33.3 / 24.7 / 20.8 / 19.4 / 20.9 us)
constexpr int kScanThreads = 512, kScanItems = 1, kScanTile = kScanThreads * kScanItems;
constexpr unsigned long long kScanAgg = 1ull << 62, kScanPre = 2ull << 62, kScanVal = (1ull << 62) - 1;

// Wave 0 of a scan block: publish tile `tile`'s aggregate, then look back with the whole
// wave -- lane l reads the word of tile (window end - l); the nearest inclusive prefix ends
// the walk -- and publish the tile's inclusive prefix.  Returns the exclusive prefix (in
// every lane).  Tile words: {flag (2 bits): 1 aggregate / 2 inclusive prefix, value (62 bits)}.
__device__ int64_t scan_lookback(unsigned long long* __restrict__ tstate, int64_t tile, int64_t agg) {
  const int lane = threadIdx.x & 63;
  if (lane == 0)
    __hip_atomic_store(&tstate[tile], (tile == 0 ? kScanPre : kScanAgg) | (unsigned long long)agg,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int64_t excl = 0;
  for (int64_t end = tile - 1; end >= 0;) {
    const int64_t p = end - lane;
    const unsigned long long w =
        p >= 0 ? __hip_atomic_load(&tstate[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kScanPre;
    const unsigned long long f = w >> 62;
    const unsigned long long pre = __ballot(f == 2), inv = __ballot(f == 0);
    const int stop = pre ? __builtin_ctzll(pre) : 64;            // first lane holding a prefix
    const unsigned long long need = stop >= 63 ? ~0ull : ((2ull << stop) - 1);
    if (inv & need) {                                              // a needed tile not published yet
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    int64_t part = lane <= stop ? (int64_t)(w & kScanVal) : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    excl += part;
    if (stop < 64) break;
    end -= 64;
  }
  if (lane == 0 && tile > 0)
    __hip_atomic_store(&tstate[tile], kScanPre | (unsigned long long)(excl + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

template <int MODE>
__global__ __launch_bounds__(kScanThreads) void k_query_scan(
    const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t Q, const int64_t* __restrict__ uptr,
    const int64_t* __restrict__ iptr, int64_t U, int64_t I, int64_t* __restrict__ out,
    unsigned long long* __restrict__ tstate, unsigned int* __restrict__ tctr, int32_t* __restrict__ flag,
    const int64_t* __restrict__ offsets, ChunkDesc* __restrict__ cdesc, int32_t* __restrict__ zero_word,
    int64_t* __restrict__ qbase, int runs, int clen, int lsh, int32_t* __restrict__ slices) {
  __shared__ int s_tile;
  __shared__ int64_t s_wave[kScanThreads / 64], s_wave2[kScanThreads / 64];
  __shared__ int64_t s_prefix, s_prefix2;
  // runs mode: per-query fill state (descriptor start, -1 = no descriptors; cost prefix;
  // list bases and lengths; output base; run length; descriptor count)
  __shared__ int64_t f_c0[MODE == 1 ? kScanTile : 1], f_cost[MODE == 1 ? kScanTile : 1];
  __shared__ int64_t f_ub[MODE == 1 ? kScanTile : 1], f_ib[MODE == 1 ? kScanTile : 1];
  __shared__ int64_t f_base[MODE == 1 ? kScanTile : 1];
  __shared__ int32_t f_du[MODE == 1 ? kScanTile : 1], f_di[MODE == 1 ? kScanTile : 1];
  __shared__ int32_t f_nq[MODE == 1 ? kScanTile : 1], f_nd[MODE == 1 ? kScanTile : 1];
  // runs mode: the tile's test items and the kRunQB after it (run heads and lengths from LDS)
  __shared__ int32_t s_qi[MODE == 1 ? kScanTile + kRunQB : 1];
  const unsigned ntiles = (unsigned)((Q + 1 + kScanTile - 1) / kScanTile);
  if (threadIdx.x == 0) s_tile = (int)atomicAdd(&tctr[0], 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t q0 = tile * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  // the list bounds (and the output base) stay in registers for the descriptor fill
  // after the look-back, instead of a second dependent qu/qi -> ptr round trip
  int64_t s_ub[kScanItems], s_du[kScanItems], s_ib[kScanItems], s_di[kScanItems], s_base[kScanItems];
  int s_nq[kScanItems];
  int64_t tsum = 0, tsum2 = 0;     // tsum2: runs mode, the descriptors' scheduling cost
  if constexpr (MODE == 1) {
    static_assert(kScanItems == 1, "one query per thread");
    if (runs) {
      const int64_t qa = tile * kScanTile + threadIdx.x;
      s_qi[threadIdx.x] = qa < Q ? qi[qa] : -1;
      if (threadIdx.x < kRunQB) {
        const int64_t qb2 = tile * kScanTile + kScanTile + threadIdx.x;
        s_qi[kScanTile + threadIdx.x] = qb2 < Q ? qi[qb2] : -1;
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int it = 0; it < kScanItems; ++it) {
    const int64_t q = q0 + it;
    int64_t x = 0;
    s_ub[it] = s_du[it] = s_ib[it] = s_di[it] = s_base[it] = 0;
    s_nq[it] = 0;
    if (q < Q) {
      if (MODE == 1 && cdesc) s_base[it] = offsets[q];
      const int32_t u = qu[q], i = qi[q];
      if (u >= 0 && u < U && i >= 0 && i < I) {
        const int64_t ub = uptr[u], ib = iptr[i];
        const int64_t du = uptr[u + 1] - ub, di = iptr[i + 1] - ib;
        s_ub[it] = ub; s_du[it] = du; s_ib[it] = ib; s_di[it] = di;
        x = MODE == 0 ? du + di : (du + kChunk - 1) / kChunk + (di + kChunk - 1) / kChunk;
        if (MODE == 1 && runs) {
          // packed {chunks (candidate slots) << 31 | work descriptors}, chunks of clen ratings:
          // the item-side chunks are work only for a run head (first query of a run of equal
          // test items, runs cut at multiples of `runs`), which scores them for the whole run
          const int tt = threadIdx.x;
          const bool head = (q % runs) == 0 || (tt > 0 ? s_qi[tt - 1] : qi[q - 1]) != i;
          s_nq[it] = 0;
          if (head) {
            int nq = 1;
            const int lim = runs - (int)(q % runs);
#pragma unroll
            for (int j = 1; j < kRunQB; ++j) {
              const bool same = j < lim && s_qi[tt + j] == i;      // -1 past the batch
              nq += (same && nq == j) ? 1 : 0;
            }
            s_nq[it] = nq;
          }
          const int64_t cu = (du + clen - 1) / clen, ci = (di + clen - 1) / clen;
          x = ((cu + ci) << 31) | (cu + (head ? ci : 0));
          tsum2 += cu * kRunUserCost + (head ? ci * (s_nq[it] + 2) : 0);
        }
      } else if (MODE == 0) {
        atomicOr(flag + 1, 1);
      }
    }
    v[it] = x;
    tsum += x;
  }
  // block scan of the per-thread sums
  int64_t inc = tsum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  int64_t inc2 = tsum2;
  if (MODE == 1 && runs) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(inc2, off);
      if (lane >= off) inc2 += y;
    }
  }
  if (lane == 63) { s_wave[wave] = inc; s_wave2[wave] = inc2; }
  __syncthreads();
  int64_t wbase = 0, agg = 0, wbase2 = 0, agg2 = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    if (w < wave) { wbase += s_wave[w]; wbase2 += s_wave2[w]; }
    agg += s_wave[w];
    agg2 += s_wave2[w];
  }
  if (wave == 0) {
    const int64_t excl = scan_lookback(tstate, tile, agg);
    // runs mode: the cost prefix on the second tile-word array
    const int64_t excl2 = (MODE == 1 && runs) ? scan_lookback(tstate + ntiles, tile, agg2) : 0;
    if (lane == 0) {
      s_prefix = excl;
      s_prefix2 = excl2;
      if (MODE == 1 && tile == 0 && zero_word) zero_word[0] = 0;   // solve's coupled-query counter
    }
  }
  __syncthreads();
  int64_t run = s_prefix + wbase + inc - tsum;
  int64_t run2 = s_prefix2 + wbase2 + inc2 - tsum2;    // cost prefix of this thread's first query
  constexpr int64_t kLo = (1ll << 31) - 1;
#pragma unroll
  for (int it = 0; it < kScanItems; ++it) {
    const int64_t q = q0 + it;
    if (q <= Q) out[q] = (MODE == 1 && runs) ? run >> 31 : run;
    if (MODE == 1 && runs && q == Q) {
      // work descriptors in all; slices in all (cost run2 in slices of lam) and the end mark
      const int64_t nw = run & kLo, ns = (run2 + (1ll << lsh) - 1) >> lsh;
      qbase[4 * Q] = nw;
      qbase[4 * Q + 1] = ns;
      if (slices) slices[ns] = (int32_t)nw;
    }
    if (MODE == 1 && qbase && q < Q) {
      // per query: {out base user, item}, {candidate slot base user, item} (k_score_mf_run)
      const int64_t du = s_du[it], cr = runs ? run >> 31 : run;
      qbase[4 * q + 0] = s_base[it];
      qbase[4 * q + 1] = s_base[it] + du;
      qbase[4 * q + 2] = cr;
      qbase[4 * q + 3] = cr + (du + clen - 1) / clen;
    }
    if (MODE == 1 && runs) {
      // runs mode: this query's descriptors are written by the whole block below
      f_c0[threadIdx.x] = run & kLo;
      f_cost[threadIdx.x] = run2;
      f_ub[threadIdx.x] = s_ub[it];
      f_ib[threadIdx.x] = s_ib[it];
      f_base[threadIdx.x] = s_base[it];
      f_du[threadIdx.x] = (int32_t)s_du[it];
      f_di[threadIdx.x] = (int32_t)s_di[it];
      f_nq[threadIdx.x] = s_nq[it];
      f_nd[threadIdx.x] = (q < Q) ? (int32_t)(v[it] & kLo) : 0;
    } else
    if (MODE == 1 && cdesc && q < Q && v[it] > 0) {
      const int64_t ub = s_ub[it], du = s_du[it], ib = s_ib[it], di = s_di[it];
      int64_t c = run;
      const int64_t base = s_base[it];
      for (int64_t st = 0; st < du; st += kChunk, ++c) {
        ChunkDesc d;
        d.list_base = ub + st;
        d.out_base = base + st;
        d.q = (int32_t)q;
        d.pos0 = (int32_t)st;
        d.len = (int32_t)(du - st < kChunk ? du - st : kChunk);
        d.side = 0;
        cdesc[c] = d;
      }
      for (int64_t st = 0; st < di; st += kChunk, ++c) {
        ChunkDesc d;
        d.list_base = ib + st;
        d.out_base = base + du + st;
        d.q = (int32_t)q;
        d.pos0 = (int32_t)(du + st);
        d.len = (int32_t)(di - st < kChunk ? di - st : kChunk);
        d.side = 1;
        cdesc[c] = d;
      }
    }
    run += v[it];
  }
  if (MODE == 1 && runs && cdesc) {
    // Block-parallel descriptor fill (runs mode): the block's descriptors are one contiguous
    // range; thread t writes descriptors t, t + 256, ... of it, finding the owning query by a
    // binary search over the per-query starts in LDS (a popular item's run head has ~20
    // descriptors: one thread writing them in turn bounded this kernel).  Descriptor j of a
    // query: user chunk j < cu (cost kRunUserCost), else item chunk j - cu (cost nq + 2); the
    // descriptor whose cost range [p, p + w) holds a slice start s << lsh starts slice s
    // (slices of a descriptor costing more than a slice are empty but the last): every
    // descriptor lands in exactly one slice.
    __syncthreads();
    const int64_t dstart = f_c0[0], dend = f_c0[kScanTile - 1] + f_nd[kScanTile - 1];
    {
      for (int64_t c = dstart + threadIdx.x; c < dend; c += kScanThreads) {
        // the owner: the last thread whose start is <= c (starts ascend; a thread with no
        // descriptors shares its start with the next one, so it is never the last such)
        int lo = 0, hi = kScanTile - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (f_c0[mid] <= c) lo = mid; else hi = mid - 1;
        }
        const int t = lo;
        const int64_t j = c - f_c0[t];
        const int32_t du = f_du[t], di = f_di[t], nq = f_nq[t];
        const int64_t cu = (du + clen - 1) / clen;
        const int64_t qq = tile * kScanTile + t;
        ChunkDesc d;
        int64_t p, w;
        if (j < cu) {
          const int64_t st = j * clen;
          d.list_base = f_ub[t] + st;
          d.out_base = f_base[t] + st;
          d.pos0 = (int32_t)st;
          d.len = (int32_t)(du - st < clen ? du - st : clen);
          d.side = 0 | (1 << 8);
          p = f_cost[t] + j * kRunUserCost;
          w = kRunUserCost;
        } else {
          const int64_t st = (j - cu) * clen;
          d.list_base = f_ib[t] + st;
          d.out_base = f_base[t] + du + st;
          d.pos0 = (int32_t)(du + st);
          d.len = (int32_t)(di - st < clen ? di - st : clen);
          d.side = 1 | (nq << 8);
          p = f_cost[t] + cu * kRunUserCost + (j - cu) * (nq + 2);
          w = nq + 2;
        }
        d.q = (int32_t)qq;
        cdesc[c] = d;
        if (slices)
          for (int64_t sl = (p + (1ll << lsh) - 1) >> lsh; (sl << lsh) < p + w; ++sl) slices[sl] = (int32_t)c;
      }
    }
  }
  // the last tile to finish resets the tile words and the counters for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    // this thread published the block's tile words: wait for those stores to be performed
    // before counting the block done, so the last block's reset cannot be overtaken by a
    // straggling publish (the outputs are read by later kernels only)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned done = atomicAdd(&tctr[1], 1u);
    if (done == ntiles - 1) {
      for (unsigned t = 0; t < (MODE == 1 && runs ? 2 * ntiles : ntiles); ++t)
        __hip_atomic_store(&tstate[t], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&tctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&tctr[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- query groups (entity-shared scoring) ----
// thread per query: rank inside its user group and its item group; per side the output
// base (offsets[q], offsets[q] + |R_u|) and candidate-slot base (coff[q], coff[q] + chunks of R_u)
__global__ void k_group_count(const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t Q,
                              const int64_t* __restrict__ uptr, const int64_t* __restrict__ iptr, int64_t U, int64_t I,
                              const int64_t* __restrict__ offsets, const int64_t* __restrict__ coff,
                              unsigned long long* __restrict__ gcnt, int32_t* __restrict__ grank,
                              int64_t* __restrict__ qbase) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  int64_t ub, du, ib, di;
  query_sides(qu, qi, q, uptr, iptr, U, I, ub, du, ib, di);
  const int32_t u = qu[q], i = qi[q];
  const bool ok = (u >= 0 && u < U && i >= 0 && i < I) && (du + di > 0);
  grank[2 * q] = ok ? (int32_t)atomicAdd(&gcnt[u], 1ull) : -1;
  grank[2 * q + 1] = ok ? (int32_t)atomicAdd(&gcnt[U + i], 1ull) : -1;
  qbase[4 * q + 0] = offsets[q];
  qbase[4 * q + 1] = offsets[q] + du;
  qbase[4 * q + 2] = coff[q];
  qbase[4 * q + 3] = coff[q] + (du + kChunk - 1) / kChunk;
}

// thread per query: place it into its user group and its item group
__global__ void k_group_fill(const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t Q, int64_t U,
                             const int64_t* __restrict__ gstart, const int32_t* __restrict__ grank,
                             int32_t* __restrict__ gq) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < Q && grank[2 * t] >= 0) {
    const int32_t u = qu[t], i = qi[t];
    gq[gstart[u] + grank[2 * t]] = (int32_t)t;
    gq[gstart[U + i] + grank[2 * t + 1]] = (int32_t)t;
  }
}

// Single-pass decoupled look-back scan over the U + I entities (users, then items) of
// the two per-entity counts of the entity-shared schedule: queries per entity (gcnt ->
// gstart) and work items per entity, ceil(deg / (cpi kChunk)) * ceil(gcnt / qb) (->
// wstart; a work item covers cpi consecutive list chunks).
// Both exclusive prefixes (and the totals at [U + I]) in one launch: no library scan, no
// count array.  tstate: two arrays of tile words (queries, work items); the last tile to
// finish re-zeroes them and the two counters.
__global__ __launch_bounds__(kScanThreads) void k_group_scan(
    unsigned long long* __restrict__ gcnt, const int64_t* __restrict__ uptr, const int64_t* __restrict__ iptr,
    int64_t U, int64_t I, int qb, int cpi, int64_t* __restrict__ gstart, int64_t* __restrict__ wstart,
    unsigned long long* __restrict__ tstate, unsigned int* __restrict__ tctr) {
  __shared__ int s_tile;
  __shared__ int64_t s_wa[kScanThreads / 64], s_wb[kScanThreads / 64];
  __shared__ int64_t s_pa, s_pb;
  const int64_t nE = U + I;
  const unsigned ntiles = (unsigned)((nE + 1 + kScanTile - 1) / kScanTile);
  if (threadIdx.x == 0) s_tile = (int)atomicAdd(&tctr[0], 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t = tile * kScanTile + threadIdx.x;
  int64_t a = 0, b = 0;
  if (t < nE) {
    a = (int64_t)gcnt[t];
    // this thread is the count's only reader here (k_item_fill takes it from gstart): leave
    // it zero for the next batch's k_group_count -- no memset on the query path
    if (a > 0) gcnt[t] = 0;
    if (a > 0) {
      const int64_t deg = t < U ? uptr[t + 1] - uptr[t] : iptr[t - U + 1] - iptr[t - U];
      b = ((deg + kChunk * cpi - 1) / (kChunk * cpi)) * ((a + qb - 1) / qb);
    }
  }
  int64_t ia = a, ib = b;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t ya = __shfl_up(ia, off), yb = __shfl_up(ib, off);
    if (lane >= off) { ia += ya; ib += yb; }
  }
  if (lane == 63) { s_wa[wave] = ia; s_wb[wave] = ib; }
  __syncthreads();
  int64_t ba = 0, bb = 0, agg_a = 0, agg_b = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    if (w < wave) { ba += s_wa[w]; bb += s_wb[w]; }
    agg_a += s_wa[w];
    agg_b += s_wb[w];
  }
  if (wave == 0) {
    const int64_t ea = scan_lookback(tstate, tile, agg_a);
    const int64_t eb = scan_lookback(tstate + ntiles, tile, agg_b);
    if (lane == 0) { s_pa = ea; s_pb = eb; }
  }
  __syncthreads();
  if (t <= nE) {
    gstart[t] = s_pa + ba + ia - a;
    wstart[t] = s_pb + bb + ib - b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // the block's tile-word stores performed before it counts itself done (see k_query_scan)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned done = atomicAdd(&tctr[1], 1u);
    if (done == ntiles - 1) {
      for (unsigned w = 0; w < 2 * ntiles; ++w)
        __hip_atomic_store(&tstate[w], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&tctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&tctr[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// thread per work item (grid-stride up to wstart[nE]): its entity by binary search over
// wstart, then {entity, chunk of the entity's list, block of the entity's query group}
__global__ void k_item_fill(const int64_t* __restrict__ wstart, const int64_t* __restrict__ gstart,
                            int64_t nE, int32_t* __restrict__ witems, int qb) {
  const int64_t total = wstart[nE];
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total;
       w += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nE - 1;     // last entity t with wstart[t] <= w
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (wstart[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const int64_t b = wstart[lo];
    const int64_t nqb = (gstart[lo + 1] - gstart[lo] + qb - 1) / qb;     // the entity's query count
    witems[3 * w] = (int32_t)lo;
    witems[3 * w + 1] = (int32_t)((w - b) / nqb);    // chunk of the entity's list
    witems[3 * w + 2] = (int32_t)((w - b) % nqb);    // block of the entity's query group
  }
}

// one workgroup per query: rel[offsets[q] + p] = R_u[p] (p < deg u), then C_i
__global__ void k_write_related(const int32_t* __restrict__ qu, const int32_t* __restrict__ qi,
                                const int64_t* __restrict__ offsets, const int64_t* __restrict__ uptr,
                                const int32_t* __restrict__ urow, const int64_t* __restrict__ iptr,
                                const int32_t* __restrict__ irow, int64_t U, int64_t I, int32_t* __restrict__ rel) {
  int64_t q = blockIdx.x;
  int32_t u = qu[q], i = qi[q];
  if (u < 0 || u >= U || i < 0 || i >= I) return;
  int64_t base = offsets[q];
  int64_t ub = uptr[u], du = uptr[u + 1] - ub;
  int64_t ib = iptr[i], di = iptr[i + 1] - ib;
  for (int64_t p = threadIdx.x; p < du; p += blockDim.x) rel[base + p] = urow[ub + p];
  for (int64_t p = threadIdx.x; p < di; p += blockDim.x) rel[base + du + p] = irow[ib + p];
}

}  // namespace

namespace {

inline unsigned bits_for(int64_t n) {
  unsigned b = 1;
  while (b < 31 && ((int64_t)1 << b) < n) ++b;
  return b;
}

inline int grid_for(int64_t n, int threads, int cap = 8192) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace

// Small-k Gram work lists of the current index: items of <= chunk list rows {entity,
// start, len, slot} (longest lists first), slot < 0 = write the Gram directly, else a
// partial slot; a combine entry {entity, first slot, n slots, 0} per split entity.
hipError_t build_gram_lists(fia_ctx* c, int64_t chunk, hipStream_t s) {
  Index& X = c->idx;
  for (int sd = 0; sd < 2; ++sd) {
    const std::vector<int64_t>& hptr = X.hptr[sd];
    std::vector<int32_t> items, comb;
    int32_t slots = 0;
    for (int32_t e : X.hord[sd]) {
      const int64_t len = hptr[(size_t)e + 1] - hptr[(size_t)e];
      const int64_t nit = len == 0 ? 1 : (len + chunk - 1) / chunk;
      if (nit > 1) comb.insert(comb.end(), {e, slots, (int32_t)nit, 0});
      for (int64_t t = 0; t < nit; ++t) {
        const int64_t st = t * chunk;
        const int64_t ln = std::min<int64_t>(chunk, len - st);
        items.insert(items.end(), {e, (int32_t)st, (int32_t)(ln < 0 ? 0 : ln), nit > 1 ? slots++ : -1});
      }
    }
    X.n_gitems[sd] = (int64_t)items.size() / 4;
    X.n_gcomb[sd] = (int64_t)comb.size() / 4;
    X.n_gslots[sd] = slots;
    if (!items.empty()) {
      FIA_HIP_TRY(X.gitems[sd].reserve(sizeof(int32_t) * items.size(), s));
      FIA_HIP_TRY(hipMemcpyAsync(X.gitems[sd].ptr, items.data(), sizeof(int32_t) * items.size(), hipMemcpyHostToDevice, s));
    }
    if (!comb.empty()) {
      FIA_HIP_TRY(X.gcomb[sd].reserve(sizeof(int32_t) * comb.size(), s));
      FIA_HIP_TRY(hipMemcpyAsync(X.gcomb[sd].ptr, comb.data(), sizeof(int32_t) * comb.size(), hipMemcpyHostToDevice, s));
    }
    FIA_HIP_TRY(hipStreamSynchronize(s));   // this side's host lists are freed at the end of the iteration
  }
  X.gchunk = chunk;
  return hipSuccess;
}

// the other-side rows of the Gram stream as byte offsets into their table (id * k * 4), in
// stream order and quad-transposed: rating 4 q + g of sub-batch d at ids[kGsSub d + 4 g + q]
// (the 16 lanes of MFMA row group g read their four quads' offsets as one 16-B word),
// kGsNoRow past the list's end
__global__ void k_gs_ids(int64_t nd, const int2* __restrict__ desc, const int32_t* __restrict__ pos,
                         const int32_t* __restrict__ other0, const int32_t* __restrict__ other1, int k,
                         uint32_t* __restrict__ ids) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nd * kGsSub;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = t / kGsSub;
    const int r = 4 * (int)(t & 3) + (int)((t >> 2) & 3);   // t % 16 = 4 g + q  ->  rating 4 q + g
    const int meta = desc[d].x;
    const int valid = meta & 31, side = (meta >> 6) & 1;
    ids[t] = r < valid ? (uint32_t)(side ? other1 : other0)[pos[d] + r] * (uint32_t)(k * 4) : kGsNoRow;
  }
}

hipError_t build_gram_stream(fia_ctx* c, int k, hipStream_t s) {
  Index& X = c->idx;
  if (X.gs_version == X.version && X.gs_k == k && X.gswave.ptr) return hipSuccess;
  struct Seg {
    int64_t len;
    int side;
    int32_t e, start, slot;
  };
  std::vector<Seg> segs;
  std::vector<int32_t> comb[2];
  for (int sd = 0; sd < 2; ++sd) {
    const std::vector<int64_t>& hptr = X.hptr[sd];
    int32_t slots = 0;
    for (int32_t e : X.hord[sd]) {
      const int64_t len = hptr[(size_t)e + 1] - hptr[(size_t)e];
      if (len <= kGsSlice) {
        segs.push_back({len, sd, e, 0, -1});
        continue;
      }
      const int64_t nit = (len + kGsSlice - 1) / kGsSlice;
      comb[sd].insert(comb[sd].end(), {e, slots, (int32_t)nit, 0});
      for (int64_t t = 0; t < nit; ++t)
        segs.push_back({std::min<int64_t>(kGsSlice, len - t * kGsSlice), sd, e, (int32_t)(t * kGsSlice), slots++});
    }
    X.n_gsslots[sd] = slots;
  }
  // longest segments first (both sides merged): the slices of the long lists start early
  std::stable_sort(segs.begin(), segs.end(), [](const Seg& a, const Seg& b) { return a.len > b.len; });
  std::vector<int2> desc;
  std::vector<int32_t> pos, wave{0};
  int cur = 0, nseg = 0;
  auto close_wave = [&]() {
    while (cur % kGsRing) {   // a multiple of the ring per wave (one ring turn per loop trip)
      desc.push_back(int2{1 << 7, -1});
      pos.push_back(0);
      ++cur;
    }
    wave.push_back((int32_t)desc.size());
    cur = 0;
    nseg = 0;
  };
  for (const Seg& g : segs) {
    const int nsb = g.len == 0 ? 1 : (int)((g.len + kGsSub - 1) / kGsSub);
    if (cur > 0 && cur + nsb > kGsMaxSub - kGsRing) close_wave();
    for (int t = 0; t < nsb; ++t) {
      const int valid = (int)std::min<int64_t>(kGsSub, g.len - (int64_t)t * kGsSub);
      const bool last = t == nsb - 1;
      const int meta = (valid < 0 ? 0 : valid) | (last ? 1 << 5 : 0) | (g.side << 6) | (g.e << 8);
      const uint32_t out = last ? ((uint32_t)g.len << 23) | (uint32_t)(g.slot + 1) : 0u;
      desc.push_back(int2{meta, (int)out});
      pos.push_back((int32_t)(X.hptr[g.side][(size_t)g.e] + g.start + (int64_t)t * kGsSub));
    }
    cur += nsb;
    if (cur >= kGsTarget || ++nseg >= kGsMaxSeg) close_wave();
  }
  if (cur > 0) close_wave();
  const int64_t nd = (int64_t)desc.size();
  X.n_gsdesc = nd;
  X.n_gsw = (int64_t)wave.size() - 1;
  FIA_HIP_TRY(X.gsdesc.reserve(sizeof(int2) * (size_t)(nd + 2), s));
  FIA_HIP_TRY(X.gsids.reserve(sizeof(int32_t) * (size_t)((nd + 2) * kGsSub), s));
  FIA_HIP_TRY(X.gswave.reserve(sizeof(int32_t) * wave.size(), s));
  DevBuf dpos;
  FIA_HIP_TRY(dpos.reserve(sizeof(int32_t) * (size_t)(nd + 1), s));
  if (nd > 0) {
    FIA_HIP_TRY(hipMemcpyAsync(X.gsdesc.ptr, desc.data(), sizeof(int2) * (size_t)nd, hipMemcpyHostToDevice, s));
    FIA_HIP_TRY(hipMemcpyAsync(dpos.ptr, pos.data(), sizeof(int32_t) * (size_t)nd, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_gs_ids, dim3(grid_for(nd * kGsSub, 256)), dim3(256), 0, s, nd, X.gsdesc.as<int2>(),
                       dpos.as<int32_t>(), X.side[0].other.as<int32_t>(), X.side[1].other.as<int32_t>(), k,
                       X.gsids.as<uint32_t>());
    FIA_HIP_TRY(hipGetLastError());
  }
  FIA_HIP_TRY(hipMemsetAsync(X.gsdesc.as<int2>() + nd, 0, sizeof(int2) * 2, s));
  FIA_HIP_TRY(hipMemcpyAsync(X.gswave.ptr, wave.data(), sizeof(int32_t) * wave.size(), hipMemcpyHostToDevice, s));
  for (int sd = 0; sd < 2; ++sd) {
    X.n_gscomb[sd] = (int64_t)comb[sd].size() / 4;
    if (!comb[sd].empty()) {
      FIA_HIP_TRY(X.gscomb[sd].reserve(sizeof(int32_t) * comb[sd].size(), s));
      FIA_HIP_TRY(hipMemcpyAsync(X.gscomb[sd].ptr, comb[sd].data(), sizeof(int32_t) * comb[sd].size(),
                                 hipMemcpyHostToDevice, s));
    }
  }
  dpos.release(s);
  FIA_HIP_TRY(hipStreamSynchronize(s));   // the host vectors go out of scope
  X.gs_version = X.version;
  X.gs_k = k;
  return hipSuccess;
}

hipError_t build_index(fia_ctx* c, int64_t N, int64_t U, int64_t I, const int32_t* user, const int32_t* item,
                       const float* rating, hipStream_t s, std::string& why) {
  Index& X = c->idx;
  X.valid = false;
  FIA_HIP_TRY(c->flag.reserve(64, s));
  FIA_HIP_TRY(hipMemsetAsync(c->flag.ptr, 0, 64, s));
  if (N > 0) {
    hipLaunchKernelGGL(k_check_ids, dim3(grid_for(N, 256)), dim3(256), 0, s, user, item, N, U, I,
                       c->flag.as<int32_t>());
    FIA_HIP_TRY(hipGetLastError());
  }
  int32_t hflag = 0;
  FIA_HIP_TRY(hipMemcpyAsync(&hflag, c->flag.ptr, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  FIA_HIP_TRY(hipStreamSynchronize(s));
  if (hflag) {
    why = "training ids out of range [0, num_users) x [0, num_items)";
    return hipErrorInvalidValue;
  }
  DevBuf keys_sorted, tmp;
  FIA_HIP_TRY(keys_sorted.reserve(sizeof(int32_t) * (size_t)(N > 0 ? N : 1), s));
  const int32_t* key_src[2] = {user, item};
  const int32_t* other_src[2] = {item, user};
  int64_t n_ent[2] = {U, I};
  for (int sd = 0; sd < 2; ++sd) {
    Side& S = X.side[sd];
    size_t nb = sizeof(int32_t) * (size_t)(N > 0 ? N : 1);
    FIA_HIP_TRY(S.row.reserve(nb, s));
    FIA_HIP_TRY(S.other.reserve(nb, s));
    FIA_HIP_TRY(S.rating.reserve(sizeof(float) * (size_t)(N > 0 ? N : 1), s));
    FIA_HIP_TRY(S.ptr.reserve(sizeof(int64_t) * (size_t)(n_ent[sd] + 1), s));
    if (N > 0) {
      unsigned eb = bits_for(n_ent[sd]);
      rocprim::counting_iterator<int32_t> iota(0);
      size_t tb = 0;
      FIA_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tb, key_src[sd], keys_sorted.as<int32_t>(), iota,
                                            S.row.as<int32_t>(), (size_t)N, 0u, eb, s));
      FIA_HIP_TRY(tmp.reserve(tb + 16, s));
      tb = tmp.bytes;
      FIA_HIP_TRY(rocprim::radix_sort_pairs(tmp.ptr, tb, key_src[sd], keys_sorted.as<int32_t>(), iota,
                                            S.row.as<int32_t>(), (size_t)N, 0u, eb, s));
      hipLaunchKernelGGL(k_gather_side, dim3(grid_for(N, 256)), dim3(256), 0, s, S.row.as<int32_t>(),
                         other_src[sd], rating, N, S.other.as<int32_t>(), S.rating.as<float>());
      FIA_HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_list_ptr, dim3((unsigned)((n_ent[sd] + 1 + 255) / 256)), dim3(256), 0, s,
                       keys_sorted.as<int32_t>(), N, n_ent[sd], S.ptr.as<int64_t>());
    FIA_HIP_TRY(hipGetLastError());
    FIA_HIP_TRY(hipStreamSynchronize(s));   // keys_sorted is reused by the next side
    // entities by list length, longest first: the Gram kernels start the long lists early
    std::vector<int64_t> hptr((size_t)n_ent[sd] + 1);
    FIA_HIP_TRY(hipMemcpyAsync(hptr.data(), S.ptr.ptr, sizeof(int64_t) * hptr.size(), hipMemcpyDeviceToHost, s));
    FIA_HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> ord((size_t)n_ent[sd]);
    for (int64_t e = 0; e < n_ent[sd]; ++e) ord[(size_t)e] = (int32_t)e;
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
      return hptr[(size_t)a + 1] - hptr[(size_t)a] > hptr[(size_t)b + 1] - hptr[(size_t)b];
    });
    X.hptr[sd] = hptr;
    FIA_HIP_TRY(X.order[sd].reserve(sizeof(int32_t) * ord.size(), s));
    FIA_HIP_TRY(hipMemcpyAsync(X.order[sd].ptr, ord.data(), sizeof(int32_t) * ord.size(), hipMemcpyHostToDevice, s));
    FIA_HIP_TRY(hipStreamSynchronize(s));
    X.hord[sd] = ord;
  }
  FIA_HIP_TRY(build_gram_lists(c, kGramChunk, s));
  keys_sorted.release(s);
  tmp.release(s);
  // pair set, load factor <= 1/2
  int64_t cap = 1024;
  while (cap < 2 * N) cap <<= 1;
  FIA_HIP_TRY(X.pkey.reserve(sizeof(unsigned long long) * (size_t)cap, s));
  FIA_HIP_TRY(X.pcnt.reserve(sizeof(int32_t) * (size_t)cap, s));
  FIA_HIP_TRY(X.psum.reserve(sizeof(double) * (size_t)cap, s));
  FIA_HIP_TRY(hipMemsetAsync(X.pkey.ptr, 0xff, sizeof(unsigned long long) * (size_t)cap, s));
  FIA_HIP_TRY(hipMemsetAsync(X.pcnt.ptr, 0, sizeof(int32_t) * (size_t)cap, s));
  FIA_HIP_TRY(hipMemsetAsync(X.psum.ptr, 0, sizeof(double) * (size_t)cap, s));
  if (N > 0) {
    hipLaunchKernelGGL(k_pair_insert, dim3(grid_for(N, 256)), dim3(256), 0, s, user, item, rating, N, I,
                       X.pkey.as<unsigned long long>(), X.pcnt.as<int32_t>(), X.psum.as<double>(),
                       (unsigned long long)(cap - 1));
    FIA_HIP_TRY(hipGetLastError());
  }
  FIA_HIP_TRY(hipStreamSynchronize(s));
  X.pcap = cap;
  ++X.version;
  X.N = N;
  X.U = U;
  X.I = I;
  X.valid = true;
  return hipSuccess;
}

// tile words + two counters of k_query_scan, zero when (re)allocated; every launch leaves
// them zero again
static hipError_t scan_state(fia_ctx* c, int64_t Q, hipStream_t s) {
  const int64_t ntiles = (Q + 1 + kScanTile - 1) / kScanTile;
  const size_t need = sizeof(unsigned long long) * (size_t)(2 * ntiles) + 16;   // two tile-word arrays (runs)
  if (c->qscan.bytes >= need && c->qscan.ptr) return hipSuccess;
  // stream-ordered regrow (the previous launches on s still own the old block)
  FIA_HIP_TRY(c->qscan.reserve(need < 4096 ? 4096 : need, s));
  FIA_HIP_TRY(hipMemsetAsync(c->qscan.ptr, 0, c->qscan.bytes, s));
  return hipSuccess;
}

template <int MODE>
static hipError_t launch_query_scan(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int64_t* out,
                                    const int64_t* offsets, ChunkDesc* cdesc, int32_t* zero_word, hipStream_t s,
                                    int64_t* qbase = nullptr, int runs = 0, int clen = kChunk, int lsh = 0,
                                    int32_t* slices = nullptr) {
  FIA_HIP_TRY(scan_state(c, Q, s));
  FIA_HIP_TRY(c->flag.reserve(64, s));
  const int64_t ntiles = (Q + 1 + kScanTile - 1) / kScanTile;
  unsigned int* ctr = reinterpret_cast<unsigned int*>(c->qscan.as<char>() + c->qscan.bytes - 16);
  // (MODE 1: the caller's phase events, if any, stamped by this dispatch)
  hipExtLaunchKernelGGL(k_query_scan<MODE>, dim3((unsigned)ntiles), dim3(kScanThreads), 0, s,
                        MODE == 1 ? c->scan_ev[0] : nullptr, MODE == 1 ? c->scan_ev[1] : nullptr, 0, qu, qi, Q,
                        c->idx.side[0].ptr.as<int64_t>(), c->idx.side[1].ptr.as<int64_t>(), c->idx.U, c->idx.I, out,
                        c->qscan.as<unsigned long long>(), ctr, c->flag.as<int32_t>(), offsets, cdesc, zero_word, qbase,
                        runs, clen, lsh, slices);
  return hipGetLastError();
}

hipError_t count_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int64_t* offsets,
                         hipStream_t s) {
  return launch_query_scan<0>(c, Q, qu, qi, offsets, nullptr, nullptr, nullptr, s);
}

hipError_t write_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                         int32_t* rel, hipStream_t s) {
  if (Q == 0) return hipSuccess;
  hipLaunchKernelGGL(k_write_related, dim3((unsigned)Q), dim3(256), 0, s, qu, qi, offsets,
                     c->idx.side[0].ptr.as<int64_t>(), c->idx.side[0].row.as<int32_t>(),
                     c->idx.side[1].ptr.as<int64_t>(), c->idx.side[1].row.as<int32_t>(), c->idx.U, c->idx.I, rel);
  return hipGetLastError();
}


hipError_t build_chunks(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                        int64_t max_chunks, bool offsets_only, hipStream_t s, int32_t* zero_word, bool runs,
                        int slice_cost, int run_chunk) {
  FIA_HIP_TRY(c->coff.reserve(sizeof(int64_t) * (size_t)(Q + 1), s));
  const bool rq = runs && !offsets_only;
  if (!offsets_only) FIA_HIP_TRY(c->cdesc.reserve(sizeof(ChunkDesc) * (size_t)(max_chunks + 1), s));
  int lsh = 0;                                   // slice cost: the power of two >= slice_cost
  while ((1 << lsh) < slice_cost && lsh < 30) ++lsh;
  const int lam = 1 << lsh;
  if (rq) {
    FIA_HIP_TRY(c->qbase.reserve(sizeof(int64_t) * (size_t)(4 * Q + 2), s));
    // total cost <= (kRunQB + 2) per descriptor
    FIA_HIP_TRY(c->slices.reserve(sizeof(int32_t) * (size_t)((max_chunks + 1) * (kRunQB + 2) / lam + 2), s));
  }
  return launch_query_scan<1>(c, Q, qu, qi, c->coff.as<int64_t>(), offsets,
                              offsets_only ? nullptr : c->cdesc.as<ChunkDesc>(), zero_word, s,
                              rq ? c->qbase.as<int64_t>() : nullptr, rq ? kRunQB : 0, rq ? run_chunk : kChunk, lsh,
                              rq ? c->slices.as<int32_t>() : nullptr);
}

hipError_t build_groups(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                        int64_t max_items, int qb, hipStream_t s, int cpi) {
  const int64_t U = c->idx.U, I = c->idx.I, nE = U + I;
  const int64_t ntiles = (nE + 1 + kScanTile - 1) / kScanTile;
  // per-entity query counts: zero at allocation, left zero by k_group_scan
  if (c->gcnt.bytes < sizeof(int64_t) * (size_t)(nE + 1) || !c->gcnt.ptr) {
    FIA_HIP_TRY(c->gcnt.reserve(sizeof(int64_t) * (size_t)(nE + 1), s));
    FIA_HIP_TRY(hipMemsetAsync(c->gcnt.ptr, 0, c->gcnt.bytes, s));
  }
  FIA_HIP_TRY(c->gstart.reserve(sizeof(int64_t) * (size_t)(nE + 1), s));
  FIA_HIP_TRY(c->wstart.reserve(sizeof(int64_t) * (size_t)(nE + 1), s));
  FIA_HIP_TRY(c->grank.reserve(sizeof(int32_t) * (size_t)(2 * Q + 1), s));
  FIA_HIP_TRY(c->gq.reserve(sizeof(int32_t) * (size_t)(2 * Q + 1), s));
  FIA_HIP_TRY(c->qbase.reserve(sizeof(int64_t) * (size_t)(4 * Q + 1), s));
  FIA_HIP_TRY(c->witems.reserve(sizeof(int32_t) * (size_t)(3 * max_items + 3), s));
  // k_group_scan state: 2 x ntiles tile words + 2 counters, zero at allocation and left zero
  const size_t need = sizeof(unsigned long long) * (size_t)(2 * ntiles) + 16;
  if (c->gscan.bytes < need || !c->gscan.ptr) {
    FIA_HIP_TRY(c->gscan.reserve(need, s));
    FIA_HIP_TRY(hipMemsetAsync(c->gscan.ptr, 0, c->gscan.bytes, s));
  }
  const int64_t* uptr = c->idx.side[0].ptr.as<int64_t>();
  const int64_t* iptr = c->idx.side[1].ptr.as<int64_t>();
  if (Q > 0) {
    hipLaunchKernelGGL(k_group_count, dim3((unsigned)((Q + 255) / 256)), dim3(256), 0, s, qu, qi, Q, uptr, iptr, U, I,
                       offsets, c->coff.as<int64_t>(), c->gcnt.as<unsigned long long>(), c->grank.as<int32_t>(),
                       c->qbase.as<int64_t>());
    FIA_HIP_TRY(hipGetLastError());
  }
  unsigned int* ctr = reinterpret_cast<unsigned int*>(c->gscan.as<char>() + c->gscan.bytes - 16);
  hipLaunchKernelGGL(k_group_scan, dim3((unsigned)ntiles), dim3(kScanThreads), 0, s, c->gcnt.as<unsigned long long>(),
                     uptr, iptr, U, I, qb, cpi, c->gstart.as<int64_t>(), c->wstart.as<int64_t>(),
                     c->gscan.as<unsigned long long>(), ctr);
  FIA_HIP_TRY(hipGetLastError());
  if (Q > 0) {
    hipLaunchKernelGGL(k_group_fill, dim3((unsigned)((Q + 255) / 256)), dim3(256), 0, s, qu, qi, Q, U,
                       c->gstart.as<int64_t>(), c->grank.as<int32_t>(), c->gq.as<int32_t>());
    FIA_HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_item_fill, dim3(grid_for(max_items, 256, 16384)), dim3(256), 0, s, c->wstart.as<int64_t>(),
                     c->gstart.as<int64_t>(), nE, c->witems.as<int32_t>(), qb);
  return hipGetLastError();
}

}  // namespace fia
