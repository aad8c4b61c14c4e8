// sg_plan.hip -- the LDS search's phase plan, built on the device.
//
// sg_sssp.hip "Bounds" / "Exact seeds": rows whose search starts from bounds
// (and exact seeds) taken from neighbour rows finished in an earlier phase.  A
// simulation computes its table once (sim_config.rs:137-141, :411-448), so the
// plan is part of every build; building it on the host cost ~6 ms against a
// 3.3 ms search at C3 (r02).  Here it is three launches on the build's stream,
// with no host work and no copy:
//
//  * k_plan_sets (one workgroup; the rows' state in LDS): phase 0 is a dominating
//    set of the rows (row u is covered by a chosen v when u == v or u has an arc
//    to v), each later phase but the last a dominating set of the rows left, the
//    last phase the rest.  Each set is a parallel greedy: in every round, each
//    live (unassigned, uncovered) row names its best candidate in its closed
//    out-neighbourhood -- most live rows in reach, then the lowest row -- and a
//    candidate joins when every live row it would cover named it.  The round's
//    joiners cover disjoint live rows, the globally best candidate always joins
//    (so a round never stalls), and the sets come out as small as the sequential
//    greedy's (C3: 1,665 rows against 1,680 in phase 0, in 26 rounds).  The row
//    lists per phase are then written in row order.
//  * k_plan_bounds (one wave per row): the row's kb best bound rows in earlier
//    phases, exact seeds first (a zero-loss arc, or a path of up to `hops`
//    zero-loss arcs), then by latency, then by row.  The zero-loss paths are
//    walked level by level, the wave's lanes taking the level's arcs in turn.
//
// The plan changes speed only, never the table: any phase assignment whose bound
// rows lie in earlier phases reaches the same fixed point (sg_sssp.hip header).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "sg_device.h"
#include "sg_internal.h"

namespace sg {

constexpr uint8_t ST_PH = 7;      // phase + 1 (0: not yet assigned)
constexpr uint8_t ST_SEL = 0x40;  // joins the current phase's set this round
constexpr uint8_t ST_COV = 0x80;  // covered in the current phase
constexpr uint32_t NO_ROW = 0xFFFFu;

// k_plan_sets keeps each row's out-neighbour rows where no round has to fetch
// them again: a thread owns the rows tid + k * NT (k < PS_RPT) for the whole
// plan and holds their first PS_REG neighbour rows in registers (u16 pairs);
// further neighbours go to an LDS pool, and a row the pool cannot take reads its
// arcs from global memory each time (rare: out-degree above PS_REG).  A round is
// then LDS work and barriers only.  (Fetching the arcs every round made each
// round ~60 us: one CU's texture path gathering scattered 12-B records.)
constexpr int PS_RPT = 11;  // rows per thread: up to 11,264 rows (the LDS search's limit is ~10.9k nodes)
constexpr int PS_REG = 8;   // neighbour rows per row held in registers
constexpr uint32_t PS_GLOBAL = 0x80000000u;  // ovf[u]: the row's arcs start at (ovf & ~PS_GLOBAL) in global memory

// LDS of k_plan_sets: gains (two u16 per word), beaten bits, node -> row u16[n], state u8[rows],
// overflow offsets u32[rows], then the pool (u16) in what is left
static size_t plan_sets_lds_fixed(uint32_t n, uint32_t rows) {
  auto al4 = [](size_t b) { return (b + 3) / 4 * 4; };
  return al4((size_t)(rows + 1) / 2 * 4) + (size_t)(rows + 31) / 32 * 4 + al4((size_t)n * 2) + al4(rows) +
         (size_t)rows * 4;
}

template <int NT>
__global__ void __launch_bounds__(NT)
    k_plan_sets(uint32_t n, const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_arc,
                uint32_t n_arcs, const uint32_t* __restrict__ used, uint32_t row_begin, uint32_t rows, int n_phase,
                uint32_t pool_cap, const uint8_t* __restrict__ given, uint32_t* __restrict__ rel_out,
                uint8_t* __restrict__ phase_out,
                uint32_t* __restrict__ list, uint32_t* __restrict__ ctl, uint32_t* __restrict__ ctr) {
  constexpr int NW = NT / 64;
  extern __shared__ __align__(16) unsigned char smem[];
  auto al4 = [](size_t b) { return (b + 3) / 4 * 4; };
  const uint32_t nwords = (rows + 31) / 32;
  unsigned char* p = smem;
  uint32_t* gain2 = (uint32_t*)p;  // live rows in a candidate's closed in-neighbourhood (arcs counted), u16 halves
  p += al4((size_t)(rows + 1) / 2 * 4);
  uint32_t* beaten = (uint32_t*)p;  // a live row in reach named another candidate this round
  p += (size_t)nwords * 4;
  uint16_t* rel16 = (uint16_t*)p;
  p += al4((size_t)n * 2);
  uint8_t* st = p;
  p += al4(rows);
  uint32_t* ovf = (uint32_t*)p;  // neighbours past PS_REG: pool offset, or PS_GLOBAL | first arc
  p += (size_t)rows * 4;
  uint16_t* pool = (uint16_t*)p;
  __shared__ uint32_t s_live, s_pool, s_wsum[NW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  for (uint32_t v = tid; v < n; v += NT) rel16[v] = (uint16_t)NO_ROW;
  for (int i = tid; i < 2 * SSSP_PHASES_MAX; i += NT) ctr[i] = 0;  // the phase launches' claim counters
  if (tid == 0) s_pool = 0;
  __syncthreads();
  for (uint32_t r = tid; r < rows; r += NT) {
    rel16[used[row_begin + r]] = (uint16_t)r;
    st[r] = 0;
  }
  __syncthreads();
  for (uint32_t v = tid; v < n; v += NT) rel_out[v] = rel16[v] == NO_ROW ? ~0u : rel16[v];
  // this thread's rows: PS_REG neighbour rows in registers (NO_ROW-padded), the degree past them
  uint32_t adj[PS_RPT][PS_REG / 2], more[PS_RPT];
#pragma unroll
  for (int k = 0; k < PS_RPT; k++) {
    const uint32_t u = tid + k * NT;
#pragma unroll
    for (int j = 0; j < PS_REG / 2; j++) adj[k][j] = 0xFFFFFFFFu;
    more[k] = 0;
    if (u >= rows) continue;
    const uint32_t v = used[row_begin + u], a0 = out_off[v], d = out_off[v + 1] - a0;
    uint32_t h[PS_REG];
#pragma unroll
    for (int j = 0; j < PS_REG; h[j] = j < (int)d ? out_arc[3 * (size_t)(a0 + j)] : 0u, j++) {
    }
#pragma unroll
    for (int j = 0; j < PS_REG; j++) {
      const uint32_t c = j < (int)d ? rel16[h[j]] : NO_ROW;
      adj[k][j / 2] = (j & 1) ? (adj[k][j / 2] & 0xFFFFu) | (c << 16) : (adj[k][j / 2] & 0xFFFF0000u) | c;
    }
    if (d > PS_REG) {
      const uint32_t m = d - PS_REG;
      more[k] = m;
      const uint32_t at = atomicAdd(&s_pool, m);
      if (at + m <= pool_cap) {
        for (uint32_t j = 0; j < m; j++) pool[at + j] = (uint16_t)rel16[out_arc[3 * (size_t)(a0 + PS_REG + j)]];
        ovf[u] = at;
      } else {
        ovf[u] = PS_GLOBAL | (a0 + PS_REG);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  auto gain = [&](uint32_t c) { return (gain2[c >> 1] >> (16 * (c & 1))) & 0xFFFFu; };
  auto gain_add = [&](uint32_t c, int d) {  // never below 0: no borrow into the other half
    atomicAdd(&gain2[c >> 1], (uint32_t)d << (16 * (c & 1)));
  };
  auto score = [&](uint32_t c) { return (gain(c) << 16) | (0xFFFFu - c); };  // most gain, then the lowest row
  // f(c) for each out-neighbour row c of this thread's k-th row u
  static_assert(PS_REG == 8, "four packed registers per row");
  auto for_out_rows = [&](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t m, uint32_t u, auto&& f) {
    const uint32_t a[4] = {a0, a1, a2, a3};  // (values: a pointer into adj[] would put it in scratch)
#pragma unroll
    for (int j = 0; j < PS_REG; j++) {
      const uint32_t c = (a[j / 2] >> (16 * (j & 1))) & 0xFFFFu;
      if (c != NO_ROW) f(c);
    }
    if (m) {
      const uint32_t o = ovf[u];
      for (uint32_t j = 0; j < m; j++) {
        const uint32_t c = (o & PS_GLOBAL) ? rel16[out_arc[3 * (size_t)((o & ~PS_GLOBAL) + j)]] : pool[o + j];
        if (c != NO_ROW) f(c);
      }
    }
  };
  auto unassigned = [&](uint32_t c) { return !(st[c] & ST_PH); };
  uint32_t named[PS_RPT];

  if (given)  // SG_PLAN_HOST (A/B diagnostics): phases computed on the host
    for (uint32_t r = tid; r < rows; r += NT) st[r] = (uint8_t)(given[r] + 1);
  for (int ph = 0; !given && ph + 1 < n_phase; ph++) {
    if (tid == 0) s_live = 0;
    for (uint32_t w = tid; w < nwords; w += NT) beaten[w] = 0;
    for (uint32_t w = tid; w < (rows + 1) / 2; w += NT) gain2[w] = 0;
    __syncthreads();
    // every unassigned row is live at the phase's start: it counts for itself and for each
    // unassigned row it has an arc to
    uint32_t nl = 0;
#pragma unroll
    for (int k = 0; k < PS_RPT; k++) {
      const uint32_t u = tid + k * NT;
      if (u >= rows || !unassigned(u)) continue;
      st[u] = 0;
      nl++;
      gain_add(u, 1);
      for_out_rows(adj[k][0], adj[k][1], adj[k][2], adj[k][3], more[k], u, [&](uint32_t c) {
        if (unassigned(c)) gain_add(c, 1);
      });
      __builtin_amdgcn_sched_barrier(0);  // one slot at a time (interleaved slots spill)
    }
    if (nl) atomicAdd(&s_live, nl);
    __syncthreads();
    for (uint32_t round = 0; s_live && round <= rows; round++) {
      // (a) each live row names its best candidate; every other candidate in its reach is beaten
#pragma unroll
      for (int k = 0; k < PS_RPT; k++) {
        const uint32_t u = tid + k * NT;
        if (u >= rows || st[u]) continue;  // assigned or covered
        uint32_t best = score(u);
        for_out_rows(adj[k][0], adj[k][1], adj[k][2], adj[k][3], more[k], u, [&](uint32_t c) {
          if (unassigned(c)) best = max(best, score(c));
        });
        const uint32_t b = 0xFFFFu - (best & 0xFFFFu);
        named[k] = b;
        if (b != u) atomicOr(&beaten[u >> 5], 1u << (u & 31));
        for_out_rows(adj[k][0], adj[k][1], adj[k][2], adj[k][3], more[k], u, [&](uint32_t c) {
          if (c != b && unassigned(c)) atomicOr(&beaten[c >> 5], 1u << (c & 31));
        });
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
      // (b) a candidate with live rows in reach, none of which named another, joins
      for (uint32_t c = tid; c < rows; c += NT)
        if (unassigned(c) && gain(c) && !((beaten[c >> 5] >> (c & 31)) & 1u)) st[c] |= ST_SEL;
      __syncthreads();
      // (c) a live row whose candidate joined is covered (the joiners' live rows are
      // disjoint), and leaves the gain of every candidate in its closed out-neighbourhood
      uint32_t ncov = 0;
#pragma unroll
      for (int k = 0; k < PS_RPT; k++) {
        const uint32_t u = tid + k * NT;
        if (u >= rows || (st[u] & (ST_PH | ST_COV)) || !(st[named[k]] & ST_SEL)) continue;
        st[u] |= ST_COV;  // (others read only the SEL bit of this byte this step)
        ncov++;
        gain_add(u, -1);
        for_out_rows(adj[k][0], adj[k][1], adj[k][2], adj[k][3], more[k], u, [&](uint32_t c) {
          if (unassigned(c)) gain_add(c, -1);
        });
        __builtin_amdgcn_sched_barrier(0);
      }
      for (uint32_t w = tid; w < nwords; w += NT) beaten[w] = 0;
      if (ncov) atomicSub(&s_live, ncov);
      __syncthreads();
      // (d) the joiners take the phase
      for (uint32_t u = tid; u < rows; u += NT)
        if (st[u] & ST_SEL) st[u] = (uint8_t)(ph + 1);
      __syncthreads();
    }
  }
  for (uint32_t r = tid; r < rows; r += NT)
    if (!(st[r] & ST_PH)) st[r] = (uint8_t)n_phase;  // the last phase: the rest
  __syncthreads();
  // the rows of each phase in row order (block-wide scans)
  uint32_t base = 0;
  for (int ph = 0; ph < n_phase; ph++) {
    const uint32_t start = base;
    for (uint32_t r0 = 0; r0 < rows; r0 += NT) {
      const uint32_t r = r0 + tid;
      const bool f = r < rows && (st[r] & ST_PH) == ph + 1;
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
  for (uint32_t r = tid; r < rows; r += NT) phase_out[r] = (uint8_t)((st[r] & ST_PH) - 1);
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
                             uint32_t row_end, int n_phase, int kb, bool exact, int hops) {
  (void)n_used;
  const uint32_t n = net->n_nodes, rows = row_end - row_begin;
  n_phase = std::max(2, std::min(SSSP_PHASES_MAX, n_phase));
  const size_t lds_fixed = plan_sets_lds_fixed(n, rows);
  constexpr size_t PS_LDS = 160 * 1024 - 64;  // (static LDS: a few words)
  if (lds_fixed + 1024 > PS_LDS || rows > (uint32_t)PS_RPT * 1024 || rows >= NO_ROW)
    throw Error(SG_ERR_INVALID_ARG, "graph too large for the device plan");
  const uint32_t pool_cap = (uint32_t)std::min<size_t>((PS_LDS - lds_fixed) / 2, 0x7FFFFFFF);
  const size_t lds = lds_fixed + (size_t)pool_cap * 2;
  // one workspace: list, ub_row, ub_w (rows x SSSP_KB_MAX each), ctl, ctr, rel (n), phase (u8 rows)
  const size_t nl = rows, nb = (size_t)rows * SSSP_KB_MAX;
  const size_t words = nl + 2 * nb + 4 * SSSP_PHASES_MAX + n + (rows + 3) / 4;
  uint32_t* w = ctx->r_plan.get<uint32_t>(words);
  SsspDevPlan p;
  p.n_phase = n_phase;
  p.list = w;
  p.ub_row = p.list + nl;
  p.ub_w = p.ub_row + nb;
  p.ctl = p.ub_w + nb;
  p.ctr = p.ctl + 2 * SSSP_PHASES_MAX;
  uint32_t* rel = p.ctr + 2 * SSSP_PHASES_MAX;
  uint8_t* phase_of = (uint8_t*)(rel + n);
  uint8_t* given = nullptr;
  if (getenv("SG_PLAN_HOST") && atoi(getenv("SG_PLAN_HOST"))) {
    // A/B diagnostics: the r02 host plan's sequential lazy greedy (bucket queue, LIFO)
    std::vector<uint32_t> off(n + 1), arc((size_t)net->n_arcs * 3), used(rows);
    copy_to_host(ctx, off.data(), net->out_off, off.size() * 4);
    copy_to_host(ctx, arc.data(), net->out_arc, arc.size() * 4);
    copy_to_host(ctx, used.data(), d_used + row_begin, rows * 4ull);
    std::vector<uint32_t> rel(n, ~0u), in_off(rows + 1, 0), in_row;
    for (uint32_t r = 0; r < rows; r++) rel[used[r]] = r;
    for (uint32_t r = 0; r < rows; r++)
      for (uint32_t a = off[used[r]]; a < off[used[r] + 1]; a++)
        if (rel[arc[3 * a]] != ~0u) in_off[rel[arc[3 * a]] + 1]++;
    for (uint32_t r = 0; r < rows; r++) in_off[r + 1] += in_off[r];
    in_row.resize(in_off[rows]);
    std::vector<uint32_t> cur(in_off.begin(), in_off.end() - 1);
    for (uint32_t r = 0; r < rows; r++)
      for (uint32_t a = off[used[r]]; a < off[used[r] + 1]; a++)
        if (rel[arc[3 * a]] != ~0u) in_row[cur[rel[arc[3 * a]]]++] = r;
    std::vector<int> phase(rows, -1);
    for (int ph = 0; ph + 1 < n_phase; ph++) {
      std::vector<uint8_t> covered(rows, 0);
      auto live = [&](uint32_t u) { return phase[u] < 0 && !covered[u]; };
      auto gain = [&](uint32_t v) {
        uint32_t g = live(v);
        for (uint32_t k = in_off[v]; k < in_off[v + 1]; k++) g += live(in_row[k]);
        return g;
      };
      std::vector<uint32_t> gn(rows, 0);
      uint32_t top = 0;
      for (uint32_t r = 0; r < rows; r++)
        if (phase[r] < 0) top = std::max(top, gn[r] = gain(r));
      std::vector<std::vector<uint32_t>> bucket(top + 1);
      for (uint32_t r = rows; r-- > 0;)
        if (phase[r] < 0 && gn[r]) bucket[gn[r]].push_back(r);
      std::vector<uint32_t> chosen;
      for (uint32_t g = top; g > 0;) {
        if (bucket[g].empty()) {
          g--;
          continue;
        }
        const uint32_t v = bucket[g].back();
        bucket[g].pop_back();
        const uint32_t gv = gain(v);
        if (gv == 0) continue;
        if (gv < g) {
          bucket[gv].push_back(v);
          continue;
        }
        chosen.push_back(v);
        covered[v] = 1;
        for (uint32_t k = in_off[v]; k < in_off[v + 1]; k++) covered[in_row[k]] = 1;
      }
      for (uint32_t v : chosen) phase[v] = ph;
    }
    std::vector<uint8_t> h8(rows);
    for (uint32_t r = 0; r < rows; r++) h8[r] = (uint8_t)(phase[r] < 0 ? n_phase - 1 : phase[r]);
    given = ctx->r_misc.get<uint8_t>(rows);
    SG_HIP(hipMemcpy(given, h8.data(), rows, hipMemcpyHostToDevice));
  }
  {
    TimedLaunch tl(ctx, "plan_sets", 0.0);
    SG_HIP(hipFuncSetAttribute((const void*)k_plan_sets<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    hipLaunchKernelGGL(k_plan_sets<1024>, dim3(1), dim3(1024), lds, ctx->stream, n, net->out_off, net->out_arc,
                       net->n_arcs, d_used, row_begin, rows, n_phase, pool_cap, given, rel, phase_of, p.list, p.ctl,
                       p.ctr);
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
