// The exact k-mer table grouped by neuron (nk_exact.h "grouped layout").
//
// The reference builds `counts` (key -> u32) and the full kmer_per_neuron in
// every process call (src/spiking_hash.rs:157-172).  Equal keys hash to the
// same neuron, so the table is built from the count's own partition instead of
// a global sort of every key:
//   K1a<KEYS>  (nk_kernels.hip) each record of a bucket region (2^13 neurons,
//              kXMinBinBits; NK_XBIN_BITS 14/15 for tests) carries its key
//              beside its bin offset;
//   k_xcount   per (bucket, slice of kXSlice records): records per group of
//              2^ggbits neurons (32 at config 2) in an LDS histogram, one row
//              per slice;
//   k_xscan    per bucket: the rows -> the offset of every (slice, group) in
//              group-major order, and each group's start;
//   k_xbase    the buckets' table bases (their records before them);
//   k_xscatter per (bucket, slice), one workgroup per CU, XCD-aware order:
//              8192-record sub-tiles counting-sorted by group in LDS, then
//              written as contiguous runs (one radix pass of at most 256
//              digits: a slice's run of a group is one stretch);
//   k_xgroup   per group, 2^gbits neurons per pass (the group's records re-read
//              from L2): an LDS hash table of 4096 slots (key -> u32 count,
//              wrapping like the reference's AtomicU32), distinct keys per
//              neuron = kmer_per_neuron, entries written neuron by neuron
//              (ent[n] = start | len << 40) into the group's own range (its
//              records' offsets: no reservation), the rest of the range
//              (duplicates) filled with (0, count 0).
// A pass whose distinct keys do not fit the LDS table, and every record of a
// bucket whose region overflowed in K1a, go to the side list instead; the host
// sorts that list (rocPRIM) and appends its run-length encoding as a key-sorted
// part (ent = kSideEnt for those neurons).  get_count scans the neuron's
// entries (grouped) or binary-searches the side part.
// (Measured and not kept, profiles/r03_*: 2048-slot tables, 4096-record
// sub-tiles, three scatter workgroups per CU, the plain workgroup order.)
#include <stdlib.h>

#include "nk_device.h"
#include "nk_exact.h"

namespace nk {

namespace {

constexpr int kXsBlock = 256;
constexpr int kXsPer = 8;                           // records per 16-B load of bins
constexpr int kXsRound = kXsBlock * kXsPer;         // 2048
constexpr int kGroupN = 1 << kXGroupBits;          // largest group
constexpr uint16_t kPadBin = 0xFFFFu;
constexpr unsigned long long kHashEmpty = ~0ull;

__device__ __forceinline__ uint64_t region_fill(const XGroupArgs &t, uint32_t b) {
  const uint64_t f = t.fill[b] & ((1ull << 40) - 1);
  return f < t.cap ? f : t.cap;
}

__device__ __forceinline__ uint32_t bucket_records(const XGroupArgs &t, uint32_t b) {
  return t.overflow[b] ? 0u : t.gstart[(uint64_t)b * (t.n_groups + 1) + t.n_groups];
}

__global__ __launch_bounds__(kXsBlock) void k_xcount(XGroupArgs t) {
  __shared__ uint32_t h[kXMaxGroups];
  const uint32_t sl = blockIdx.x, b = blockIdx.y, NG = t.n_groups;
  const uint64_t fill = region_fill(t, b);
  const uint64_t r0 = (uint64_t)sl * kXSlice;
  if (t.overflow[b] || r0 >= fill) return;  // (k_xscan reads only the rows of used slices)
  if (threadIdx.x < NG) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t r1 = fill < r0 + kXSlice ? fill : r0 + kXSlice;  // both multiples of 8
  const uint16_t *off = t.off + (uint64_t)b * t.cap;
  for (uint64_t r = r0 + (uint64_t)threadIdx.x * kXsPer; r < r1; r += kXsRound) {
    const uint4 v = *reinterpret_cast<const uint4 *>(off + r);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo = w[i] & 0xFFFFu, hi = w[i] >> 16;
      if (lo != kPadBin) atomicAdd(&h[lo >> t.ggbits], 1u);
      if (hi != kPadBin) atomicAdd(&h[hi >> t.ggbits], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < NG) t.xcnt[((uint64_t)b * t.n_slices + sl) * NG + threadIdx.x] = h[threadIdx.x];
}

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_w, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t i = 0; i < wv; ++i) pre += s_w[i];
  *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  __syncthreads();
  return pre + x - v;
}

// one workgroup per bucket, one thread per group: rows [slice][group] ->
// absolute offsets in the bucket's regrouped region (group-major)
__global__ __launch_bounds__(kXsBlock) void k_xscan(XGroupArgs t) {
  __shared__ uint32_t s_w[4];
  const uint32_t b = blockIdx.x, NG = t.n_groups, g = threadIdx.x;
  const uint64_t fill = region_fill(t, b);
  const uint32_t used = t.overflow[b] ? 0u : (uint32_t)((fill + kXSlice - 1) / kXSlice);
  uint32_t *row0 = t.xcnt + (uint64_t)b * t.n_slices * NG + g;
  uint32_t run = 0;
  if (g < NG)
    for (uint32_t sl = 0; sl < used; ++sl) {
      const uint32_t v = row0[(uint64_t)sl * NG];
      row0[(uint64_t)sl * NG] = run;
      run += v;
    }
  uint32_t total;
  const uint32_t start = block_excl_scan(run, s_w, &total);
  uint32_t *gst = t.gstart + (uint64_t)b * (NG + 1);
  if (g < NG) {
    gst[g] = start;
    for (uint32_t sl = 0; sl < used; ++sl) row0[(uint64_t)sl * NG] += start;
  }
  if (g == 0) gst[NG] = total;
}

// the buckets' table bases: exclusive scan of their records (one block)
__global__ __launch_bounds__(512) void k_xbase(XGroupArgs t) {
  __shared__ unsigned long long s[512];
  const uint32_t b = threadIdx.x;
  const unsigned long long v = b < t.n_buckets ? bucket_records(t, b) : 0ull;
  s[b] = v;
  __syncthreads();
  for (int o = 1; o < 512; o <<= 1) {  // Hillis-Steele, inclusive
    const unsigned long long y = b >= (uint32_t)o ? s[b - o] : 0ull;
    __syncthreads();
    s[b] += y;
    __syncthreads();
  }
  if (b < t.n_buckets) {
    t.bbase[b] = s[b] - v;
    t.bdist[b] = 0;
  }
  if (b == 511) *t.span = s[511];
}

// per (bucket, slice): 4096-record sub-tiles counting-sorted by group in LDS,
// each group's records appended to its run (cursor from the scan); a side
// bucket's records go to the side list
// XCD-aware order: workgroups are placed on the 8 XCDs round-robin by their
// linear index, so linear index L runs on XCD L % 8; bucket b's slices all go
// to XCD b % 8, one after another, so the adjacent pieces of a group's runs
// that consecutive slices write meet in one L2
constexpr int kSub = 8192;  // records per LDS sub-tile
__global__ __launch_bounds__(kXsBlock) void k_xscatter(XGroupArgs t) {
  constexpr int kSubPer = kSub / kXsBlock;  // per thread
  __shared__ unsigned long long s_key[kSub];
  __shared__ uint8_t s_bin[kSub], s_grp[kSub];
  __shared__ uint32_t cnt[kXMaxGroups], st[kXMaxGroups], gcur[kXMaxGroups], s_w[4];
  __shared__ unsigned long long s_at;
  __shared__ uint32_t s_n;
  const uint32_t L = blockIdx.x, x = L & 7u, kk = L >> 3;
  const uint32_t b = x + 8u * (kk / t.n_slices), sl = kk % t.n_slices;
  if (b >= t.n_buckets) return;
  const uint32_t NG = t.n_groups, tid = threadIdx.x;
  const uint64_t fill = region_fill(t, b);
  const uint64_t r0 = (uint64_t)sl * kXSlice;
  if (r0 >= fill) return;
  const uint64_t r1 = fill < r0 + kXSlice ? fill : r0 + kXSlice;
  const uint64_t base = (uint64_t)b * t.cap;
  const uint16_t *off = t.off + base;
  const uint64_t *key = t.key + base;
  if (t.overflow[b]) {  // side bucket: every record's key to the side list
    for (uint64_t rr = r0; rr < r1; rr += kXsRound) {  // uniform trip count (barriers inside)
      const uint64_t r = rr + (uint64_t)tid * kXsPer;
      uint32_t n = 0;
      uint16_t o[kXsPer];
      if (r < r1) {
        const uint4 v = *reinterpret_cast<const uint4 *>(off + r);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o[2 * i] = (uint16_t)(w[i] & 0xFFFFu);
          o[2 * i + 1] = (uint16_t)(w[i] >> 16);
        }
#pragma unroll
        for (int i = 0; i < kXsPer; ++i) n += o[i] != kPadBin;
      }
      if (tid == 0) s_n = 0;
      __syncthreads();
      const uint32_t my = n ? atomicAdd(&s_n, n) : 0u;
      __syncthreads();
      if (tid == 0) s_at = s_n ? atomicAdd(t.n_side, (unsigned long long)s_n) : 0ull;
      __syncthreads();
      unsigned long long at = s_at + my;
      if (n)
        for (int i = 0; i < kXsPer; ++i)
          if (o[i] != kPadBin) {
            if (at < t.side_cap) t.side[at] = key[r + i];
            ++at;
          }
      __syncthreads();
    }
    return;
  }
  if (tid < NG) gcur[tid] = t.xcnt[((uint64_t)b * t.n_slices + sl) * NG + tid];
  uint64_t *key2 = t.key2 + base;
  uint8_t *bin2 = t.bin2 + base;
  // this thread's 16 records of a sub-tile: s0 + j * 2048 + tid * 8 + i (16-B
  // loads contiguous across the wave); the bins and keys of the next sub-tile
  // are loaded while this one is sorted and written
  constexpr int kJ = kSubPer / kXsPer;  // 16-B loads of bins per thread and sub-tile
  uint4 vo[kJ];
  ulonglong2 vk[kJ][kXsPer / 2];
  auto load_sub = [&](uint64_t s0) {
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const uint64_t r = s0 + (uint64_t)j * kXsRound + (uint64_t)tid * kXsPer;
      const bool in = r < r1;
      vo[j] = in ? *reinterpret_cast<const uint4 *>(off + r)
                 : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
#pragma unroll
      for (int i = 0; i < kXsPer / 2; ++i)
        vk[j][i] = in ? *reinterpret_cast<const ulonglong2 *>(key + r + 2 * i) : make_ulonglong2(0, 0);
    }
  };
  load_sub(r0);
  for (uint64_t s0 = r0; s0 < r1; s0 += kSub) {
    uint4 co[kJ];
    ulonglong2 ck[kJ][kXsPer / 2];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      co[j] = vo[j];
#pragma unroll
      for (int i = 0; i < kXsPer / 2; ++i) ck[j][i] = vk[j][i];
    }
    if (s0 + kSub < r1) load_sub(s0 + kSub);
    if (tid < NG) cnt[tid] = 0;
    __syncthreads();
    // (group, neuron in group, rank) of each record
    uint32_t gr[kSubPer];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const uint32_t w[4] = {co[j].x, co[j].y, co[j].z, co[j].w};
#pragma unroll
      for (int i = 0; i < kXsPer; ++i) {
        const uint32_t o = (i & 1) ? (w[i >> 1] >> 16) : (w[i >> 1] & 0xFFFFu);
        uint32_t x = 0xFFFFFFFFu;
        if (o != kPadBin) {
          const uint32_t g = o >> t.ggbits;
          x = (g << 24) | ((o & ((1u << t.ggbits) - 1u)) << 16) | atomicAdd(&cnt[g], 1u);
        }
        gr[j * kXsPer + i] = x;
      }
    }
    __syncthreads();
    uint32_t total;
    const uint32_t mine = tid < NG ? cnt[tid] : 0u;
    const uint32_t pre = block_excl_scan(mine, s_w, &total);
    if (tid < NG) st[tid] = pre;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
#pragma unroll
      for (int i = 0; i < kXsPer; ++i) {
        const uint32_t x = gr[j * kXsPer + i];
        if (x == 0xFFFFFFFFu) continue;
        const uint32_t p = st[x >> 24] + (x & 0xFFFFu);
        s_key[p] = (i & 1) ? ck[j][i >> 1].y : ck[j][i >> 1].x;
        s_bin[p] = (uint8_t)((x >> 16) & 0xFFu);
        s_grp[p] = (uint8_t)(x >> 24);
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < total; i += kXsBlock) {  // runs: consecutive i, consecutive dst
      const uint32_t g = s_grp[i];
      const uint32_t d = gcur[g] + (i - st[g]);
      key2[d] = s_key[i];
      bin2[d] = s_bin[i];
    }
    __syncthreads();
    if (tid < NG) gcur[tid] += cnt[tid];
  }
}

// one workgroup per group of 2^ggbits neurons; 2^gbits neurons per LDS pass.
// A slot's count word holds the neuron (bits 25..31) and the count (bits
// 0..24), which cannot overflow below 2^25 records per group.
constexpr uint32_t kCntBits = 25;
constexpr uint32_t kCntMask = (1u << kCntBits) - 1u;
constexpr int kXgBatch = 8;   // records per thread in flight
constexpr int kMaxProbe = 128;  // a longer probe sends the pass to the side list

// a batch of the group's records: kp / bp = the group's first record (launch-
// uniform per workgroup), i0 + u * 256 + tid < n the records of this batch
__device__ __forceinline__ void xg_load(const uint64_t *kp, const uint8_t *bp, uint32_t i0, uint32_t n,
                                        uint32_t (&bn)[kXgBatch],
                                        uint64_t (&ky)[kXgBatch]) {
#pragma unroll
  for (int u = 0; u < kXgBatch; ++u) {
    const uint32_t i = i0 + (uint32_t)u * kXsBlock + threadIdx.x;
    bn[u] = i < n ? (uint32_t)bp[i] : 0xFFu;
  }
#pragma unroll
  for (int u = 0; u < kXgBatch; ++u) {
    const uint32_t i = i0 + (uint32_t)u * kXsBlock + threadIdx.x;
    // not predicated on the bin just loaded (that made the key loads a second
    // dependent round trip); another pass's records are filtered at insert
    ky[u] = i < n ? kp[i] : 0ull;
  }
}

// 4096-slot LDS table (48 KB with its counts): three workgroups per CU
__global__ __launch_bounds__(kXsBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_xgroup(XGroupArgs t) {
  constexpr int kHashBits = 12, kHashSlots = 1 << kHashBits, kSlotsPer = kHashSlots / kXsBlock;
  constexpr uint32_t kHashMax = kHashSlots * 5 / 8;
  __shared__ unsigned long long hk[kHashSlots];
  __shared__ uint32_t hc[kHashSlots];
  __shared__ uint32_t bc[kGroupN], bcur[kGroupN], spc[kGroupN], s_w[4];
  __shared__ uint32_t s_fail;
  const uint32_t g = blockIdx.x, b = blockIdx.y, NG = t.n_groups, tid = threadIdx.x;
  const uint64_t n0 = ((uint64_t)b << t.bin_bits) + ((uint64_t)g << t.ggbits);
  if (n0 >= t.pool) return;
  const uint32_t nG = (uint32_t)(t.pool - n0 < (uint64_t)(1u << t.ggbits) ? t.pool - n0 : (1u << t.ggbits));
  if (t.overflow[b]) {  // side bucket
    if (tid < nG) {
      t.ent[n0 + tid] = kSideEnt;
      t.kpn[n0 + tid] = 0;
    }
    return;
  }
  const uint32_t *gst = t.gstart + (uint64_t)b * (NG + 1);
  const uint64_t base = (uint64_t)b * t.cap;
  const uint64_t gs = base + gst[g], ge = base + gst[g + 1];
  const uint32_t hmax = t.hash_max && t.hash_max < kHashMax ? t.hash_max : kHashMax;
  const uint32_t W = 1u << t.gbits;  // neurons per pass
  const bool big = ge - gs >= (uint64_t)kCntMask;
  const unsigned long long tbase = t.bbase[b] + gst[g];  // this group's table range
  unsigned long long used = 0;                            // entries written so far
  for (uint32_t p0 = 0; p0 < nG; p0 += W) {
    const uint32_t pn = nG - p0 < W ? nG - p0 : W;  // neurons of this pass
#pragma unroll
    for (int i = 0; i < kSlotsPer; ++i) hk[tid + i * kXsBlock] = kHashEmpty;
#pragma unroll
    for (int i = 0; i < kSlotsPer; ++i) hc[tid + i * kXsBlock] = 0;
    if (tid < kGroupN) bc[tid] = spc[tid] = 0;
    if (tid == 0) s_fail = 0;
    __syncthreads();
    // the pass's records, kXgBatch per thread in flight (all loads of a batch
    // issued before the first insert); the first probe of 8 records at a time
    // as independent LDS CAS (one return latency for all 8), the rare
    // collisions probed on one by one.  No count field can overflow: a group
    // of 2^25 records or more goes to the side list whole (big).
    const uint64_t *kp = t.key2 + gs;
    const uint8_t *bp = t.bin2 + gs;
    const uint32_t nrec = (uint32_t)(ge - gs);
    for (uint32_t i0 = 0; i0 < nrec && !big; i0 += kXsBlock * kXgBatch) {
      uint32_t cb[kXgBatch];
      uint64_t ck[kXgBatch];
      xg_load(kp, bp, i0, nrec, cb, ck);
      if (*(volatile uint32_t *)&s_fail) break;
#pragma unroll
      for (int u0 = 0; u0 < kXgBatch; u0 += 8) {
        uint32_t hh[8];
        unsigned long long pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint64_t key = ck[u0 + u];
          hh[u] = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - kHashBits));
          pv[u] = (cb[u0 + u] - p0 < pn && key != kHashEmpty)
                      ? atomicCAS(&hk[hh[u]], kHashEmpty, (unsigned long long)key)
                      : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint32_t bin = cb[u0 + u];
          if (bin - p0 >= pn) continue;  // another pass's neuron (or past the group)
          const uint64_t key = ck[u0 + u];
          if (key == kHashEmpty) {  // only k = 32 non-canonical (all T): kept beside the table
            atomicAdd(&spc[bin], 1u);
            continue;
          }
          unsigned long long prev = pv[u];
          uint32_t h = hh[u];
          for (int probe = 1; prev != kHashEmpty && prev != key; ++probe) {
            if (probe == kMaxProbe) {
              s_fail = 1u;
              break;
            }
            h = (h + 1) & (kHashSlots - 1);
            prev = atomicCAS(&hk[h], kHashEmpty, (unsigned long long)key);
          }
          // u32 count field; the neuron is added in by the slot's first insert
          if (prev == kHashEmpty) atomicAdd(&hc[h], 1u | (bin << kCntBits));
          else if (prev == key) atomicAdd(&hc[h], 1u);
        }
      }
    }    __syncthreads();
    // distinct keys per neuron of the pass
    unsigned long long rk[kSlotsPer];
    uint32_t rc[kSlotsPer];
    if (!s_fail) {
#pragma unroll
      for (int i = 0; i < kSlotsPer; ++i) {
        const int sidx = tid + i * kXsBlock;
        rk[i] = hk[sidx];
        rc[i] = hc[sidx];
        if (rk[i] != kHashEmpty) atomicAdd(&bc[rc[i] >> kCntBits], 1u);
      }
    }
    __syncthreads();
    const uint32_t nb = p0 + tid;  // one neuron per thread (tid < pn)
    const uint32_t len = tid < pn ? bc[nb] + (spc[nb] ? 1u : 0u) : 0u;
    uint32_t D;
    const uint32_t pre = block_excl_scan(len, s_w, &D);
    if (big || s_fail || D > hmax) {  // too many distinct keys for the LDS table: this pass to the side list
      if (tid < pn) {
        t.ent[n0 + p0 + tid] = kSideEnt;
        t.kpn[n0 + p0 + tid] = 0;
      }
      const uint32_t lane = tid & 63;
      for (uint64_t r0 = gs; r0 < ge; r0 += kXsBlock) {
        const uint64_t r = r0 + tid;
        const bool take = r < ge && t.bin2[r] - p0 < pn;
        const uint64_t m = __ballot(take);
        unsigned long long at = 0;
        if (lane == 0 && m) at = atomicAdd(t.n_side, (unsigned long long)__popcll(m));
        at = __shfl(at, 0, 64) + __popcll(m & ((1ull << lane) - 1ull));
        if (take && at < t.side_cap) t.side[at] = t.key2[r];
      }
      __syncthreads();
      continue;
    }
    const unsigned long long at = tbase + used;
    used += D;
    if (tid < pn) {
      bcur[nb] = pre;
      t.ent[n0 + nb] = (at + pre) | ((unsigned long long)len << 40);
      t.kpn[n0 + nb] = len;  // kmer_per_neuron (src/spiking_hash.rs:167-172)
    }
    __syncthreads();
    // entries -> LDS in neuron order (the ~0 key, the largest, last in its neuron)
#pragma unroll
    for (int i = 0; i < kSlotsPer; ++i)
      if (rk[i] != kHashEmpty) {
        const uint32_t q = atomicAdd(&bcur[rc[i] >> kCntBits], 1u);
        hk[q] = rk[i];
        hc[q] = rc[i] & kCntMask;
      }
    __syncthreads();
    if (tid < pn && spc[nb]) {
      hk[bcur[nb]] = kHashEmpty;
      hc[bcur[nb]] = spc[nb];
    }
    __syncthreads();
    for (uint32_t i = tid; i < D; i += kXsBlock) {
      t.uniq[at + i] = hk[i];
      t.cnt[at + i] = hc[i];
    }
    __syncthreads();
  }
  // the rest of the group's range: (0, count 0); its distinct keys to the bucket
  for (unsigned long long i = tbase + used + tid; i < tbase + (ge - gs); i += kXsBlock) {
    t.uniq[i] = 0;
    t.cnt[i] = 0;
  }
  if (tid == 0 && used) atomicAdd(&t.bdist[b], used);
}

// the entry counts: one block over the buckets
__global__ __launch_bounds__(256) void k_xfinish(XGroupArgs t, unsigned long long *n,
                                                 const unsigned long long *n_side_uniq) {
  __shared__ unsigned long long s[256];
  unsigned long long d = 0;
  for (uint32_t b = threadIdx.x; b < t.n_buckets; b += 256) d += t.bdist[b];
  s[threadIdx.x] = d;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < (uint32_t)o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const unsigned long long sp = *t.span, u = n_side_uniq ? *n_side_uniq : 0ull;
    n[0] = sp + u;
    n[1] = sp;
    n[5] = s[0] + u;
  }
}

}  // namespace

uint32_t xgroup_hash_bits() { return 12; }

uint32_t xgroup_bits(uint64_t n_records, uint64_t pool) {
  // about (table slots) / 2 distinct keys per pass at most (a neuron's records
  // bound its distinct keys)
  const double per = pool ? (double)n_records / (double)pool : 0.0;
  const double half = (double)(1u << xgroup_hash_bits()) / 2;
  uint32_t gb = kXGroupBits;
  while (gb > 0 && (double)(1u << gb) * per > half) --gb;
  return gb;
}

bool xgroup_fits(uint64_t n_records, uint64_t pool, uint32_t gbits) {
  const double per = pool ? (double)n_records / (double)pool : 0.0;
  return (double)(1u << gbits) * per <= (double)((1u << xgroup_hash_bits()) * 5 / 8) * 0.8;
}

hipError_t xgroup_build(const XGroupArgs &t, hipStream_t s) {
  if (!t.n_buckets) return hipSuccess;
  if (t.n_buckets > 512 || t.ggbits > (uint32_t)kXGroupBits || t.bin_bits < t.ggbits ||
      t.bin_bits > 15 || t.gbits > t.ggbits || t.n_groups != (1u << (t.bin_bits - t.ggbits)) ||
      t.n_groups > (uint32_t)kXMaxGroups || t.cap >= (1ull << 32))
    return hipErrorInvalidValue;
  const dim3 gs(t.n_slices, t.n_buckets);
  hipLaunchKernelGGL(k_xcount, gs, dim3(kXsBlock), 0, s, t);
  hipLaunchKernelGGL(k_xscan, dim3(t.n_buckets), dim3(kXsBlock), 0, s, t);
  hipLaunchKernelGGL(k_xbase, dim3(1), dim3(512), 0, s, t);
  // one k_xscatter workgroup per CU: each keeps ~512 group runs with a partial
  // 128-B line open in L2 (keys and bins), and three per CU overflowed the
  // XCD's L2 with them (exact step 2.97-2.99 ms with 3 per CU, 2.98-3.06 with
  // 2, 2.92-2.94 with 1 -- 80 KB of unused dynamic LDS --, profiles/r03_xspad);
  // the LDS one workgroup per CU may use holds 8192-record sub-tiles, runs
  // twice as long (2.92-2.94 vs 2.94-2.95 ms, profiles/r03_xssub)
  hipLaunchKernelGGL(k_xscatter, dim3(8u * ((t.n_buckets + 7u) / 8u) * t.n_slices), dim3(kXsBlock),
                     0, s, t);
  hipLaunchKernelGGL(k_xgroup, dim3(t.n_groups, t.n_buckets), dim3(kXsBlock), 0, s, t);
  return hipGetLastError();
}

hipError_t xgroup_finish(const XGroupArgs &t, unsigned long long *n,
                         const unsigned long long *n_side_uniq, hipStream_t s) {
  hipLaunchKernelGGL(k_xfinish, dim3(1), dim3(256), 0, s, t, n, n_side_uniq);
  return hipGetLastError();
}

}  // namespace nk
