// sg_plan.hip -- the LDS search's phase plan, built on the device.
//
// sg_sssp.hip "Bounds" / "Exact seeds": rows whose search starts from bounds
// (and exact seeds) taken from neighbour rows finished in an earlier phase.  A
// simulation computes its table once (sim_config.rs:137-141, :411-448), so the
// plan is part of every build; building it on the host cost ~6 ms against a
// 3.3 ms search at C3 (r02).  Here it is a few grid-wide launches on the build's
// stream, with no host work and no copy:
//
//  * Phase sets by vote (k_vote_gain, k_vote_name; two launches per set): every
//    row not yet in a phase names its best candidate in its closed out-
//    neighbourhood (itself and the rows it has an arc to) -- the one with the
//    most such rows in its closed in-neighbourhood, then the lowest row -- and
//    every named row joins the phase.  A set so made dominates the rows left (each
//    named a member it reaches), so every row of a later phase has a bound row.
//    Phase 0 comes out 1.5x the size of a greedy dominating set (C3: 2,561 rows
//    against 1,665), but the greedy needs ~26 dependent rounds per set, and in one
//    workgroup those cost 1.1 ms against the 0.2 ms the smaller first phase
//    saves; and the later phases, bounded by the larger sets, search faster: the
//    searches of both plans take the same 3.2 ms (tools/sssp_ab.py, one box).
//  * k_plan_lists (one workgroup): each phase's rows in row order, the counts.
//  * k_plan_bounds (one wave per row): the row's kb best bound rows in earlier
//    phases, exact seeds first (a zero-loss arc, or a path of up to `hops`
//    zero-loss arcs), then by latency, then by row.  The zero-loss paths are
//    walked level by level, the wave's lanes taking the level's arcs in turn.
//
//  * Landmarks (undirected graphs): phase 0's rows run from infinity, about twice
//    as long as a bounded row.  So phase 0 is split: n_land of its rows, spread
//    evenly over it, run first (one claim round of the persistent workgroups); the
//    rest of phase 0 then starts from bounds through the nearest landmarks L,
//    D[s][v] <= D[s][L] + D[L][v] with D[s][L] = D[L][s].latency -- the reversed
//    path L -> s has the same latency in an undirected graph (petgraph keeps both
//    arc directions, graph/mod.rs:137-152).  Latency bounds only, never exact
//    seeds (the reversed path's loss fold differs).  k_plan_landmarks relabels the
//    phases; sssp_landmark_bounds (a launch between phases 0 and 1) reads D[L][s]
//    from the landmark rows just written and keeps each row's kb nearest.
//
// The plan changes speed only, never the table: any phase assignment whose bound
// rows lie in earlier phases reaches the same fixed point (sg_sssp.hip header).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

// rel[used row] = its relative row; also zeroes jn (and the caller's per-row flags):
// no fills on the build's path
__global__ void k_plan_rel(const uint32_t* __restrict__ used, uint32_t row_begin, uint32_t rows,
                           uint32_t* __restrict__ rel, uint8_t* __restrict__ jn, uint32_t* __restrict__ zero_rows,
                           uint32_t* __restrict__ zero_rows2) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  rel[used[row_begin + r]] = r;
  jn[r] = 0;
  if (zero_rows) zero_rows[r] = 0;
  if (zero_rows2) zero_rows2[r] = 0;
}

// jn[r]: 0 while row r is in no phase, else its phase + 1 (set once).  Gain of an
// unassigned row c for the set of phase ph: the unassigned rows in its closed
// in-neighbourhood (arcs counted).
// The vote kernels take a row's arcs eight at a time with branch-free buffer loads
// (an out-of-range offset reads 0, no traffic): each step is one chain of dependent
// loads (arc -> rel -> jn / gain) with eight arcs in flight, not eight chains in turn.
constexpr uint32_t PL_OOB = 0x80000000u;
constexpr int PL_ARCS = 8;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pl_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7FFFFFFF, 0x00020000);
}

__global__ void k_vote_gain(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_idx,
                            uint32_t in_stride, const uint32_t* __restrict__ used, uint32_t row_begin, uint32_t rows,
                            const uint32_t* __restrict__ rel, const uint8_t* __restrict__ jn,
                            uint32_t* __restrict__ gain) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= rows || jn[c]) return;
  const uint32_t v = used[row_begin + c];
  const __amdgpu_buffer_rsrc_t ri = pl_rsrc(in_idx), rr = pl_rsrc(rel), rj = pl_rsrc(jn);
  const uint32_t a0 = in_off[v], a1 = in_off[v + 1];
  uint32_t g = 1;
  for (uint32_t a = a0; a < a1; a += PL_ARCS) {
    uint32_t t[PL_ARCS], u[PL_ARCS];
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++)
      t[k] = __builtin_amdgcn_raw_buffer_load_b32(ri, a + k < a1 ? (a + k) * in_stride * 4u : PL_OOB, 0, 0);
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++) u[k] = __builtin_amdgcn_raw_buffer_load_b32(rr, a + k < a1 ? t[k] * 4u : PL_OOB, 0, 0);
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++) {
      const bool on = a + k < a1 && u[k] != ~0u;
      const uint8_t x = __builtin_amdgcn_raw_buffer_load_b8(rj, on ? u[k] : PL_OOB, 0, 0);
      g += on && !x;
    }
  }
  gain[c] = g;
}

// Each unassigned row names its best candidate, which joins phase ph.  A candidate
// that joins during this launch still counts as unassigned here (jn == ph + 1).
__global__ void k_vote_name(const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc,
                            const uint32_t* __restrict__ used, uint32_t row_begin, uint32_t rows,
                            const uint32_t* __restrict__ rel, uint8_t* __restrict__ jn,
                            const uint32_t* __restrict__ gain, int ph) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= rows) return;
  const uint8_t tag = (uint8_t)(ph + 1);
  auto open_tag = [&](uint8_t x) { return x == 0 || x == tag; };
  if (!open_tag(jn[u])) return;  // in an earlier phase (a row named during this launch still names)
  auto score = [&](uint32_t g, uint32_t c) { return ((uint64_t)g << 32) | (0xFFFFFFFFu - c); };
  const uint32_t v = used[row_begin + u];
  uint64_t best = score(gain[u], u);
  const __amdgpu_buffer_rsrc_t ra = pl_rsrc(out_arc), rr = pl_rsrc(rel), rj = pl_rsrc(jn), rg = pl_rsrc(gain);
  const uint32_t a0 = out_off[v], a1 = out_off[v + 1];
  for (uint32_t a = a0; a < a1; a += PL_ARCS) {
    uint32_t t[PL_ARCS], c[PL_ARCS], g[PL_ARCS];
    uint8_t x[PL_ARCS];
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++)
      t[k] = __builtin_amdgcn_raw_buffer_load_b32(ra, a + k < a1 ? (a + k) * 12u : PL_OOB, 0, 0);
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++) c[k] = __builtin_amdgcn_raw_buffer_load_b32(rr, a + k < a1 ? t[k] * 4u : PL_OOB, 0, 0);
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++) {
      const bool on = a + k < a1 && c[k] != ~0u;
      x[k] = __builtin_amdgcn_raw_buffer_load_b8(rj, on ? c[k] : PL_OOB, 0, 0);
      g[k] = __builtin_amdgcn_raw_buffer_load_b32(rg, on ? c[k] * 4u : PL_OOB, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < PL_ARCS; k++)
      if (a + k < a1 && c[k] != ~0u && open_tag(x[k])) best = max(best, score(g[k], c[k]));
  }
  jn[0xFFFFFFFFu - (uint32_t)best] = tag;
}

// Landmarks: n_land rows of phase 0 (jn == 1), evenly spread over its rows in row
// order, stay in phase 0; every other row assigned a phase moves one phase later.
template <int NT>
__global__ void __launch_bounds__(NT) k_plan_landmarks(uint8_t* __restrict__ jn, uint32_t rows, uint32_t n_land) {
  constexpr int NW = NT / 64;
  __shared__ uint32_t s_wsum[NW];
  __shared__ uint32_t s_total;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t cnt = 0;  // phase-0 rows
  for (uint32_t r = tid; r < rows; r += NT) cnt += jn[r] == 1;
  for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
  if (lane == 0) s_wsum[wv] = cnt;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (int w = 0; w < NW; w++) t += s_wsum[w];
    s_total = t;
  }
  __syncthreads();
  const uint32_t s0 = s_total;
  uint32_t base = 0;  // phase-0 rows before this pass's chunk
  for (uint32_t r0 = 0; r0 < rows; r0 += NT) {
    const uint32_t r = r0 + tid;
    const uint8_t x = r < rows ? jn[r] : 0;
    const bool f = x == 1;
    const uint32_t incl = wave_incl_sum(f ? 1u : 0u);
    __syncthreads();  // s_wsum reuse
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int w = 0; w < NW; w++) {
      pre += w < wv ? s_wsum[w] : 0u;
      tot += s_wsum[w];
    }
    if (r < rows && x) {
      bool land = false;
      if (f && n_land < s0) {  // index i among phase 0: a landmark where floor(i * n_land / s0) steps
        const uint64_t i = base + pre + incl - 1;
        land = i == 0 || (i * n_land) / s0 != ((i - 1) * n_land) / s0;
      }
      jn[r] = land ? 1 : (uint8_t)(x + 1);
    }
    base += tot;
  }
}

// Phase 1's bound rows: for each of its rows s, the kb landmarks L nearest to s
// by D[L][s] (column s of the landmark rows, just written by phase 0), as
// latency-only bounds with w = D[L][s].  A landmark row that gave up (sat_row 2)
// was never written and is skipped.
constexpr int LB_MAX = 4;
__global__ void __launch_bounds__(256)
    k_landmark_bounds(const uint32_t* __restrict__ list, const uint32_t* __restrict__ ctl, uint32_t n_used,
                      uint32_t row_begin, const uint64_t* __restrict__ out_lat, const uint32_t* __restrict__ sat_row,
                      int kb, uint32_t* __restrict__ ub_row, uint32_t* __restrict__ ub_w) {
  const uint32_t n_land = ctl[1], base = ctl[2], n1 = ctl[3];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n1) return;
  const uint32_t srow = list[base + i];
  uint64_t t[LB_MAX];  // (distance << 32) | landmark position, ascending
#pragma unroll
  for (int j = 0; j < LB_MAX; j++) t[j] = ~0ull;
  for (uint32_t k = 0; k < n_land; k++) {
    const uint32_t L = list[k];
    if (sat_row[L - row_begin] == 2u) continue;
    const uint64_t d = out_lat[(size_t)(L - row_begin) * n_used + srow];
    if (d >= LAT32_SAT) continue;
    uint64_t key = (d << 32) | k;
#pragma unroll
    for (int j = 0; j < LB_MAX; j++) {
      const uint64_t lo = min(t[j], key);
      key = max(t[j], key);
      t[j] = lo;
    }
  }
  // k_plan_bounds' entries for this row (landmarks it has an arc to, exact seeds
  // first) stay; the nearest landmarks fill the slots left, up to kb in all
  uint32_t* orow = ub_row + (size_t)(base + i) * SSSP_KB_MAX;
  uint32_t* ow = ub_w + (size_t)(base + i) * SSSP_KB_MAX;
  int have = 0;
  while (have < kb && orow[have] != ~0u) have++;
  int j = 0;
  for (int slot = have; slot < kb; slot++) {
    while (j < LB_MAX && t[j] != ~0ull) {  // skip a landmark already listed
      bool dup = false;
      const uint32_t L = list[(uint32_t)t[j]];
      for (int q = 0; q < have; q++) dup |= (orow[q] & ~SSSP_UB_EXACT) == L;
      if (!dup) break;
      j++;
    }
    if (j >= LB_MAX || t[j] == ~0ull) break;
    orow[slot] = list[(uint32_t)t[j]];
    ow[slot] = (uint32_t)(t[j] >> 32);
    j++;
  }
}

void sssp_landmark_bounds(sg_ctx* ctx, const SsspDevPlan& p, uint32_t n_used, uint32_t row_begin,
                          const uint64_t* out_lat, const uint32_t* sat_row, int kb) {
  // phase 1 holds at most the block's rows: one thread each, those past its count (ctl[3]) exit
  hipLaunchKernelGGL(k_landmark_bounds, dim3(p.rows_grid), dim3(256), 0, ctx->stream, p.list, p.ctl, n_used, row_begin,
                     out_lat, sat_row, std::max(1, std::min(LB_MAX, kb)), p.ub_row, p.ub_w);
  SG_CHECK_LAUNCH();
}

// Rows still in no phase take the last one; each phase's rows in row order and the
// counts; the phase launches' claim counters zeroed.  Two passes over the rows, no
// barrier inside either: (1) per (chunk of NT rows, wave, phase) counts by ballot
// into LDS; one block scan of the counts in (phase, chunk, wave) order; (2) each row
// at its (phase, chunk, wave) offset plus its rank among the wave's lanes of its
// phase.  (The earlier form scanned the rows once per phase, two barriers per chunk:
// 22 us at C3.)  Up to PL_CHUNKS chunks; larger plans take the per-phase form.
constexpr uint32_t PL_CHUNKS = 64;
template <int NT>
__global__ void __launch_bounds__(NT)
    k_plan_lists(const uint8_t* __restrict__ jn, uint32_t rows, uint32_t row_begin, int n_phase,
                 uint8_t* __restrict__ phase_out, uint32_t* __restrict__ list, uint32_t* __restrict__ ctl,
                 uint32_t* __restrict__ ctr) {
  constexpr int NW = NT / 64;
  __shared__ uint32_t s_cnt[SSSP_PHASES_MAX * PL_CHUNKS * NW];  // (phase, chunk, wave) counts, then offsets
  __shared__ uint32_t s_wsum[NW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < 2 * SSSP_PHASES_MAX; i += NT) ctr[i] = 0;
  auto phase_of = [&](uint32_t r) { return jn[r] ? (int)jn[r] - 1 : n_phase - 1; };
  const uint32_t chunks = (rows + NT - 1) / NT;
  const uint64_t lt = (1ull << lane) - 1;
  if (chunks <= PL_CHUNKS) {
    const uint32_t n_ent = (uint32_t)n_phase * chunks * NW;
    // the first PL_REG chunks' jn loaded up front (branch-free, all in flight) and kept
    // in registers for pass 2; the loops over them are unrolled (static register indices)
    constexpr uint32_t PL_REG = 16;
    uint8_t jr[PL_REG];
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc((void*)jn, 0, (int)rows, 0x00020000);
#pragma unroll
    for (uint32_t c = 0; c < PL_REG; c++) {
      const uint32_t r = c * NT + tid;
      jr[c] = __builtin_amdgcn_raw_buffer_load_b8(rj, c < chunks && r < rows ? r : 0x80000000u, 0, 0);
    }
    auto count_chunk = [&](uint32_t c, int ph) {
      for (int p = 0; p < n_phase; p++) {
        const uint64_t m = __ballot(ph == p);
        if (lane == 0) s_cnt[((uint32_t)p * chunks + c) * NW + wv] = (uint32_t)__popcll(m);
      }
      const uint32_t r = c * NT + tid;
      if (r < rows) phase_out[r] = (uint8_t)ph;
    };
#pragma unroll
    for (uint32_t c = 0; c < PL_REG; c++) {
      const uint32_t r = c * NT + tid;
      if (c < chunks) count_chunk(c, r < rows ? (jr[c] ? (int)jr[c] - 1 : n_phase - 1) : -1);
    }
    for (uint32_t c = PL_REG; c < chunks; c++) {
      const uint32_t r = c * NT + tid;
      count_chunk(c, r < rows ? phase_of(r) : -1);
    }
    __syncthreads();
    // exclusive scan of the n_ent counts: thread t sums a contiguous range of `per`
    const uint32_t per = (n_ent + NT - 1) / NT, b = tid * per, e = min(b + per, n_ent);
    uint32_t sum = 0;
    for (uint32_t i = b; i < e; i++) sum += s_cnt[i];
    const uint32_t incl = wave_incl_sum(sum);
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int w = 0; w < wv; w++) run += s_wsum[w];
    for (uint32_t i = b; i < e; i++) {
      const uint32_t x = s_cnt[i];
      s_cnt[i] = run;
      run += x;
    }
    __syncthreads();
    if (tid < n_phase) {
      const uint32_t start = chunks ? s_cnt[(uint32_t)tid * chunks * NW] : 0u;
      const uint32_t next = tid + 1 < n_phase ? s_cnt[(uint32_t)(tid + 1) * chunks * NW] : rows;
      ctl[2 * tid] = start;
      ctl[2 * tid + 1] = next - start;
    }
    auto place_chunk = [&](uint32_t c, int ph) {
      uint64_t mine = 0;
      for (int p = 0; p < n_phase; p++) {
        const uint64_t m = __ballot(ph == p);
        if (ph == p) mine = m;
      }
      const uint32_t r = c * NT + tid;
      if (r < rows) list[s_cnt[((uint32_t)ph * chunks + c) * NW + wv] + (uint32_t)__popcll(mine & lt)] = row_begin + r;
    };
#pragma unroll
    for (uint32_t c = 0; c < PL_REG; c++) {
      const uint32_t r = c * NT + tid;
      if (c < chunks) place_chunk(c, r < rows ? (jr[c] ? (int)jr[c] - 1 : n_phase - 1) : -1);
    }
    for (uint32_t c = PL_REG; c < chunks; c++) {
      const uint32_t r = c * NT + tid;
      place_chunk(c, r < rows ? phase_of(r) : -1);
    }
    return;
  }
  uint32_t base = 0;
  for (int ph = 0; ph < n_phase; ph++) {
    const uint32_t start = base;
    for (uint32_t r0 = 0; r0 < rows; r0 += NT) {
      const uint32_t r = r0 + tid;
      const bool f = r < rows && phase_of(r) == ph;
      const uint32_t incl = wave_incl_sum(f ? 1u : 0u);
      if (lane == 63) s_wsum[wv] = incl;
      __syncthreads();
      uint32_t pre = 0, tot = 0;
      for (int w = 0; w < NW; w++) {
        const uint32_t x = s_wsum[w];
        pre += w < wv ? x : 0u;
        tot += x;
      }
      if (f) list[base + pre + incl - 1] = row_begin + r;
      base += tot;
      __syncthreads();
    }
    if (tid == 0) {
      ctl[2 * ph] = start;
      ctl[2 * ph + 1] = base - start;
    }
  }
  for (uint32_t r = tid; r < rows; r += NT) phase_out[r] = (uint8_t)phase_of(r);
}

// Bound rows.  Candidate key: (not exact) << 63 | latency << 31 | relative row, so
// the u64 order is the plan's rank (exact seeds, then latency, then row).
constexpr int PB_WAVES = 4;
constexpr int PB_FMAX = 256;  // zero-loss frontier entries per wave and level (more are dropped: fewer seeds)
constexpr int PB_LIST = 4;    // candidates a lane keeps

__global__ void __launch_bounds__(PB_WAVES * 64)
    k_plan_bounds(const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc,
                  const uint32_t* __restrict__ used, const uint32_t* __restrict__ rel,
                  const uint8_t* __restrict__ phase_of, const uint32_t* __restrict__ list, uint32_t rows,
                  uint32_t row_begin, int kb, int exact, int hops, uint32_t* __restrict__ ub_row,
                  uint32_t* __restrict__ ub_w) {
  __shared__ uint32_t fx[PB_WAVES][2][PB_FMAX], fw[PB_WAVES][2][PB_FMAX], fpre[PB_WAVES][PB_FMAX + 1];
  __shared__ uint32_t fcnt[PB_WAVES][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * PB_WAVES + wv;
  if (i >= rows) return;
  const uint32_t row = list[i];
  const int ph = phase_of[row - row_begin];
  uint32_t* orow = ub_row + (size_t)i * SSSP_KB_MAX;
  uint32_t* ow = ub_w + (size_t)i * SSSP_KB_MAX;
  if (lane < SSSP_KB_MAX) {
    orow[lane] = ~0u;
    ow[lane] = 0u;
  }
  if (ph == 0) return;
  const uint32_t s = used[row];
  uint64_t t[PB_LIST];
#pragma unroll
  for (int j = 0; j < PB_LIST; j++) t[j] = ~0ull;
  auto offer = [&](uint64_t key) {  // sorted insertion, unrolled (no dynamic register indexing)
#pragma unroll
    for (int j = 0; j < PB_LIST; j++) {
      const uint64_t lo = min(t[j], key);
      key = max(t[j], key);
      t[j] = lo;
    }
  };
  // arc a at path depth `level` after w0 ns of zero-loss path; zero-loss continuations go to frontier `dst`
  auto visit = [&](uint32_t a, uint64_t w0, int level, int dst) {
    const uint32_t h = out_arc[3 * (size_t)a], l = out_arc[3 * (size_t)a + 1];
    const bool z = out_arc[3 * (size_t)a + 2] == 0x3F800000u;  // 1f32 - loss == 1.0: a zero-loss arc
    const uint64_t w = w0 + l;
    if (w >= LAT32_SAT) return;
    if (level > 1 && (!z || h == s)) return;  // past the first arc, only zero-loss paths (exact seeds)
    const uint32_t q = rel[h];
    if (q != ~0u && phase_of[q] < ph)
      offer(((uint64_t)!(exact && z) << 63) | (w << 31) | q);
    if (exact && z && level < hops && h != s) {
      const uint32_t k = atomicAdd(&fcnt[wv][dst], 1u);
      if (k < PB_FMAX) {
        fx[wv][dst][k] = h;
        fw[wv][dst][k] = (uint32_t)w;
      }
    }
  };
  if (lane == 0) {
    fcnt[wv][0] = 0;
    fcnt[wv][1] = 0;
  }
  __builtin_amdgcn_wave_barrier();
  {  // level 1: the row's own arcs
    const uint32_t a0 = out_off[s], a1 = out_off[s + 1];
    for (uint32_t a = a0 + lane; a < a1; a += 64) visit(a, 0, 1, 0);
  }
  int cur = 0;
  for (int level = 2; level <= hops; level++) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t m = min<uint32_t>(fcnt[wv][cur], PB_FMAX);
    if (!m) break;
    // arcs of the frontier entries, laid end to end: prefix of their out-degrees
    uint32_t carry = 0;
    for (uint32_t e0 = 0; e0 < m; e0 += 64) {
      const uint32_t e = e0 + lane;
      const uint32_t d = e < m ? out_off[fx[wv][cur][e] + 1] - out_off[fx[wv][cur][e]] : 0u;
      const uint32_t incl = wave_incl_sum(d);
      if (e < m) fpre[wv][e] = carry + incl - d;
      carry += __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) {
      fpre[wv][m] = carry;
      fcnt[wv][cur ^ 1] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t tt = lane; tt < carry; tt += 64) {
      uint32_t lo = 0, hi = m;  // the entry e with fpre[e] <= tt < fpre[e + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (fpre[wv][mid] <= tt) lo = mid;
        else hi = mid;
      }
      visit(out_off[fx[wv][cur][lo]] + (tt - fpre[wv][lo]), fw[wv][cur][lo], level, cur ^ 1);
    }
    cur ^= 1;
  }
  // the kb best distinct rows over the wave: repeated wave minima, each row taken once
  for (int k = 0; k < kb; k++) {
    uint64_t mk = t[0];
    for (int d = 32; d > 0; d >>= 1) mk = min(mk, (uint64_t)__shfl_xor((unsigned long long)mk, d));
    if (mk == ~0ull) break;
    const uint32_t q = (uint32_t)mk & 0x7FFFFFFFu;
    if (lane == 0) {
      orow[k] = (row_begin + q) | ((mk >> 63) ? 0u : SSSP_UB_EXACT);
      ow[k] = (uint32_t)(mk >> 31);
    }
#pragma unroll
    for (int j = 0; j < PB_LIST; j++)
      if (((uint32_t)t[j] & 0x7FFFFFFFu) == q) t[j] = ~0ull;
    // re-sort the lane's list (removed entries are ~0)
#pragma unroll
    for (int p = 0; p < PB_LIST; p++)
#pragma unroll
      for (int j = 0; j + 1 < PB_LIST; j++) {
        const uint64_t lo = min(t[j], t[j + 1]), hi = max(t[j], t[j + 1]);
        t[j] = lo;
        t[j + 1] = hi;
      }
  }
}

SsspDevPlan sssp_device_plan(sg_ctx* ctx, sg_net* net, const uint32_t* d_used, uint32_t n_used, uint32_t row_begin,
                             uint32_t row_end, int n_phase, int kb, bool exact, int hops, uint32_t n_land,
                             uint32_t* zero_rows, uint32_t* zero_rows2) {
  (void)n_used;
  const uint32_t n = net->n_nodes, rows = row_end - row_begin;
  n_phase = std::max(2, std::min(SSSP_PHASES_MAX - (n_land ? 1 : 0), n_phase));
  // one workspace: list, ub_row, ub_w (rows x SSSP_KB_MAX each), ctl, ctr, rel (n), gain (rows),
  // jn and phase (u8 rows each)
  const size_t nl = rows, nb = (size_t)rows * SSSP_KB_MAX;
  const size_t words = nl + 2 * nb + 4 * SSSP_PHASES_MAX + n + rows + 2 * ((rows + 3) / 4);
  uint32_t* w = ctx->r_plan.get<uint32_t>(words);
  SsspDevPlan p;
  p.n_phase = n_phase;
  p.list = w;
  p.ub_row = p.list + nl;
  p.ub_w = p.ub_row + nb;
  p.ctl = p.ub_w + nb;
  p.ctr = p.ctl + 2 * SSSP_PHASES_MAX;
  uint32_t* rel = p.ctr + 2 * SSSP_PHASES_MAX;
  uint32_t* gain = rel + n;
  uint8_t* jn = (uint8_t*)(gain + rows);
  uint8_t* phase_of = jn + (rows + 3) / 4 * 4;
  hipStream_t st = ctx->stream;
  {
    TimedLaunch tl(ctx, "plan_sets", 0.0);
    // rel of a node outside the block's rows reads ~0; a block of all n rows writes every entry
    if (rows != n) SG_HIP(hipMemsetAsync(rel, 0xff, (size_t)n * 4, st));
    const unsigned g = grid_for(rows, 256);
    hipLaunchKernelGGL(k_plan_rel, dim3(g), dim3(256), 0, st, d_used, row_begin, rows, rel, jn, zero_rows, zero_rows2);
    // in-neighbours: the CSC when directed; the out-arcs themselves when undirected
    if (net->directed) ensure_csc(ctx, net);
    const uint32_t* in_off = net->directed ? net->in_off : net->out_off;
    const uint32_t* in_idx = net->directed ? net->in_src : net->out_arc;
    const uint32_t in_stride = net->directed ? 1u : 3u;
    for (int ph = 0; ph + 1 < n_phase; ph++) {
      hipLaunchKernelGGL(k_vote_gain, dim3(g), dim3(256), 0, st, in_off, in_idx, in_stride, d_used, row_begin, rows,
                         rel, jn, gain);
      hipLaunchKernelGGL(k_vote_name, dim3(g), dim3(256), 0, st, net->out_off, net->out_arc, d_used, row_begin, rows,
                         rel, jn, gain, ph);
    }
    if (n_land) {  // phase 0 split: its landmark rows first (see the header)
      hipLaunchKernelGGL(k_plan_landmarks<1024>, dim3(1), dim3(1024), 0, st, jn, rows, n_land);
      n_phase += 1;
      p.n_phase = n_phase;
      p.landmarks = true;
      p.rows_grid = grid_for(rows, 256);
    }
    hipLaunchKernelGGL(k_plan_lists<1024>, dim3(1), dim3(1024), 0, st, jn, rows, row_begin, n_phase, phase_of, p.list,
                       p.ctl, p.ctr);
    SG_CHECK_LAUNCH();
  }
  {
    TimedLaunch tl(ctx, "plan_bounds", 0.0);
    hipLaunchKernelGGL(k_plan_bounds, dim3((rows + PB_WAVES - 1) / PB_WAVES), dim3(PB_WAVES * 64), 0, ctx->stream,
                       net->out_off, net->out_arc, d_used, rel, phase_of, p.list, rows, row_begin,
                       std::max(1, std::min(SSSP_KB_MAX, kb)), exact ? 1 : 0, std::max(1, std::min(3, hops)),
                       p.ub_row, p.ub_w);
    SG_CHECK_LAUNCH();
  }
  if (getenv("SG_PLAN_DIAG") && atoi(getenv("SG_PLAN_DIAG"))) {  // phase sizes on stderr
    uint32_t h[2 * SSSP_PHASES_MAX];
    copy_to_host(ctx, h, p.ctl, sizeof(h));
    fprintf(stderr, "[plan] %u rows:", rows);
    for (int ph = 0; ph < n_phase; ph++) fprintf(stderr, " %u", h[2 * ph + 1]);
    fprintf(stderr, "\n");
  }
  return p;
}

}  // namespace sg
