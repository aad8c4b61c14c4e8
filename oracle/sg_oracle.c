/*
 * sg_oracle.c -- CPU restatement of Shadow's network-core hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * implementation in shadow_amd/csrc.  Only tests/, __graft_entry__.smoke()
 * and bench.py's `cpu_baseline` leg may load it.  The product path never
 * links or calls it (and fails loudly when the HIP library is missing).
 *
 * Parity pinning: the reference (Rust, Shadow 3.2.0) cannot be built here
 * (no cargo/rustc; petgraph / rand / rand_xoshiro not vendored -- SURVEY §8c).
 * This restatement is pinned by
 *   - graph/mod.rs:564-651 test_shortest_path (9 exact latencies x {directed,
 *     undirected}) and graph/mod.rs:519-533 test_path_add,
 *   - configuration.rs:1366-1380 ONE_GBIT_SWITCH_GRAPH -> {(0,0): (1 ms, 0.0)},
 *   - the upstream rand_xoshiro 0.7.0 known-answer vector for xoshiro256++
 *     (state [1,2,3,4]) [external, restated from the published algorithm],
 *   - networkx/scipy shortest-path latencies on random graphs (tests/).
 * The f32 loss bits, the f64 draw and the event order follow the cited code;
 * the reference's own tests do not pin them ("parity unpinned" for those
 * bits beyond the restatement -- see DESIGN.md §Oracle).
 *
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off: one rounding per f32 op,
 * no FMA, matching Rust's f32 arithmetic in graph/mod.rs:328).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* Runs fn(args + t * stride) for t in [0, n) on n threads.  A thread that cannot be created runs
 * its share on the calling thread instead, and only the threads that started are joined (no join
 * of an uninitialised handle).  Shared by sg_faithful.c. */
void sgo_run_threads(void* (*fn)(void*), void* args, size_t stride, uint32_t n) {
  pthread_t* th = (pthread_t*)malloc((size_t)(n ? n : 1) * sizeof(pthread_t));
  uint8_t* ok = (uint8_t*)calloc(n ? n : 1, 1);
  for (uint32_t t = 0; t < n; t++) {
    void* a = (char*)args + (size_t)t * stride;
    if (th && ok && pthread_create(&th[t], NULL, fn, a) == 0) ok[t] = 1;
    else fn(a);
  }
  for (uint32_t t = 0; t < n; t++)
    if (ok && ok[t]) pthread_join(th[t], NULL);
  free(th);
  free(ok);
}

#define SGO_OK 0
#define SGO_ERR_NO_EDGE 1     /* graph/mod.rs:266-268 "No edge connecting node" */
#define SGO_ERR_MULTI_EDGE 2  /* graph/mod.rs:269-275 "More than one edge connecting" */
#define SGO_ERR_UNREACHABLE 3 /* graph/mod.rs:219 assert_eq!(paths.len(), n^2) panics */
#define SGO_ERR_OOM 4
#define SGO_ERR_ARG 5

/* ------------------------------------------------------------------------- */
/* PathProperties semiring (graph/mod.rs:297-340)                            */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint64_t lat;
  float loss;
} sgo_pp;

/* graph/mod.rs:322-331: (lat + lat, 1f32 - (1f32 - a) * (1f32 - b)).  Each
 * f32 op rounds once; -ffp-contract=off keeps the product from fusing. */
static inline sgo_pp pp_add(sgo_pp a, uint64_t e_lat, float e_loss) {
  sgo_pp r;
  r.lat = a.lat + e_lat; /* release-build Rust wraps; latencies never get near 2^64 */
  float oma = 1.0f - a.loss;
  float ome = 1.0f - e_loss;
  float prod = oma * ome;
  r.loss = 1.0f - prod;
  return r;
}

/* graph/mod.rs:305-313: latency first, then packet loss (f32 partial_cmp). */
static inline int pp_lt(sgo_pp a, sgo_pp b) {
  return a.lat < b.lat || (a.lat == b.lat && a.loss < b.loss);
}

void sgo_path_add(uint64_t a_lat, float a_loss, uint64_t b_lat, float b_loss, uint64_t* out_lat,
                  float* out_loss) {
  sgo_pp a = {a_lat, a_loss};
  sgo_pp r = pp_add(a, b_lat, b_loss);
  *out_lat = r.lat;
  *out_loss = r.loss;
}

/* ------------------------------------------------------------------------- */
/* Adjacency as petgraph sees it (graph/mod.rs:134-181).                      */
/* Directed: one arc per GML edge.  Undirected: both directions, a self-loop  */
/* is iterated once (petgraph Edges::next skips the second copy).             */
/* ------------------------------------------------------------------------- */
typedef struct {
  uint32_t n;
  uint32_t* off; /* n+1 */
  uint32_t* dst; /* arcs */
  uint32_t* edge; /* GML edge index of each arc */
} sgo_adj;

static void adj_free(sgo_adj* a) {
  free(a->off);
  free(a->dst);
  free(a->edge);
}

static int adj_build(sgo_adj* a, uint32_t n, uint32_t m, const uint32_t* esrc, const uint32_t* edst,
                     int directed) {
  a->n = n;
  a->off = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
  size_t cap = directed ? m : 2 * (size_t)m;
  a->dst = (uint32_t*)malloc((cap ? cap : 1) * sizeof(uint32_t));
  a->edge = (uint32_t*)malloc((cap ? cap : 1) * sizeof(uint32_t));
  if (!a->off || !a->dst || !a->edge) return SGO_ERR_OOM;
  for (uint32_t i = 0; i < m; i++) {
    if (esrc[i] >= n || edst[i] >= n) return SGO_ERR_ARG;
    a->off[esrc[i] + 1]++;
    if (!directed && esrc[i] != edst[i]) a->off[edst[i] + 1]++;
  }
  for (uint32_t v = 0; v < n; v++) a->off[v + 1] += a->off[v];
  uint32_t* cur = (uint32_t*)malloc(((size_t)n + 1) * sizeof(uint32_t));
  if (!cur) return SGO_ERR_OOM;
  memcpy(cur, a->off, ((size_t)n + 1) * sizeof(uint32_t));
  for (uint32_t i = 0; i < m; i++) {
    uint32_t s = esrc[i], d = edst[i];
    a->dst[cur[s]] = d;
    a->edge[cur[s]++] = i;
    if (!directed && s != d) {
      a->dst[cur[d]] = s;
      a->edge[cur[d]++] = i;
    }
  }
  free(cur);
  return SGO_OK;
}

/* ------------------------------------------------------------------------- */
/* petgraph 0.8.1 algo::dijkstra restated (call sites graph/mod.rs:195,198): */
/* binary heap, lazy insertion, skip visited targets, update on strict '<',  */
/* start score = PathProperties::default().                                  */
/* ------------------------------------------------------------------------- */
typedef struct {
  sgo_pp key;
  uint32_t node;
} heap_item;

typedef struct {
  heap_item* a;
  size_t n, cap;
} heap_t;

static inline int heap_less(const heap_item* x, const heap_item* y) { return pp_lt(x->key, y->key); }

static int heap_push(heap_t* h, sgo_pp key, uint32_t node) {
  if (h->n == h->cap) {
    size_t nc = h->cap ? 2 * h->cap : 1024;
    heap_item* na = (heap_item*)realloc(h->a, nc * sizeof(heap_item));
    if (!na) return SGO_ERR_OOM;
    h->a = na;
    h->cap = nc;
  }
  size_t i = h->n++;
  heap_item it = {key, node};
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!heap_less(&it, &h->a[p])) break;
    h->a[i] = h->a[p];
    i = p;
  }
  h->a[i] = it;
  return SGO_OK;
}

static heap_item heap_pop(heap_t* h) {
  heap_item top = h->a[0];
  heap_item last = h->a[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    const heap_item* best = &last;
    if (l < h->n && heap_less(&h->a[l], best)) { m = l; best = &h->a[l]; }
    if (r < h->n && heap_less(&h->a[r], best)) { m = r; best = &h->a[r]; }
    if (m == i) break;
    h->a[i] = h->a[m];
    i = m;
  }
  if (h->n) h->a[i] = last;
  return top;
}

typedef struct {
  const sgo_adj* adj;
  const uint64_t* elat;
  const float* eloss;
  const uint32_t* used;
  uint32_t n_used;
  uint64_t* out_lat;
  float* out_loss;
  uint32_t row_begin, row_end;
  int64_t next_row; /* shared work counter */
  pthread_mutex_t mu;
  int err;
  uint32_t err_row, err_col;
} sssp_job;

static int dijkstra_row(sssp_job* J, uint32_t row, sgo_pp* score, uint8_t* has, uint8_t* visited,
                        heap_t* h) {
  const sgo_adj* A = J->adj;
  uint32_t n = A->n, src = J->used[row];
  memset(has, 0, n);
  memset(visited, 0, n);
  h->n = 0;
  sgo_pp zero = {0, 0.0f};
  score[src] = zero;
  has[src] = 1;
  if (heap_push(h, zero, src)) return SGO_ERR_OOM;
  while (h->n) {
    heap_item it = heap_pop(h);
    uint32_t u = it.node;
    if (visited[u]) continue;
    for (uint32_t k = A->off[u]; k < A->off[u + 1]; k++) {
      uint32_t v = A->dst[k];
      if (visited[v]) continue;
      uint32_t e = A->edge[k];
      sgo_pp cand = pp_add(it.key, J->elat[e], J->eloss[e]);
      if (!has[v] || pp_lt(cand, score[v])) {
        score[v] = cand;
        has[v] = 1;
        if (heap_push(h, cand, v)) return SGO_ERR_OOM;
      }
    }
    visited[u] = 1;
  }
  size_t base = (size_t)(row - J->row_begin) * J->n_used;
  for (uint32_t j = 0; j < J->n_used; j++) {
    uint32_t d = J->used[j];
    if (!has[d]) {
      pthread_mutex_lock(&J->mu);
      if (J->err == 0 || row < J->err_row || (row == J->err_row && j < J->err_col)) {
        J->err = SGO_ERR_UNREACHABLE;
        J->err_row = row;
        J->err_col = j;
      }
      pthread_mutex_unlock(&J->mu);
      J->out_lat[base + j] = UINT64_MAX;
      J->out_loss[base + j] = 0.0f;
      continue;
    }
    J->out_lat[base + j] = score[d].lat;
    J->out_loss[base + j] = score[d].loss;
  }
  return SGO_OK;
}

static void* sssp_worker(void* arg) {
  sssp_job* J = (sssp_job*)arg;
  uint32_t n = J->adj->n;
  sgo_pp* score = (sgo_pp*)malloc((size_t)n * sizeof(sgo_pp) + 1);
  uint8_t* has = (uint8_t*)malloc((size_t)n + 1);
  uint8_t* visited = (uint8_t*)malloc((size_t)n + 1);
  heap_t h = {0, 0, 0};
  int rc = (!score || !has || !visited) ? SGO_ERR_OOM : SGO_OK;
  while (rc == SGO_OK) {
    int64_t row = __atomic_fetch_add(&J->next_row, 1, __ATOMIC_RELAXED);
    if (row >= (int64_t)J->row_end) break;
    rc = dijkstra_row(J, (uint32_t)row, score, has, visited, &h);
  }
  if (rc == SGO_ERR_OOM) {
    pthread_mutex_lock(&J->mu);
    J->err = SGO_ERR_OOM;
    pthread_mutex_unlock(&J->mu);
  }
  free(score);
  free(has);
  free(visited);
  free(h.a);
  return NULL;
}

/* Number of GML edges connecting u->v as petgraph edges_connecting counts them
 * (graph/mod.rs:256-293); *first receives the first such edge in adjacency order. */
static uint32_t count_connecting(const sgo_adj* A, uint32_t u, uint32_t v, uint32_t* first) {
  uint32_t c = 0;
  for (uint32_t k = A->off[u]; k < A->off[u + 1]; k++)
    if (A->dst[k] == v) {
      if (c == 0) *first = A->edge[k];
      c++;
    }
  return c;
}

/*
 * NetworkGraph::compute_shortest_paths (graph/mod.rs:183-228), dense output:
 *   out[(i - row_begin) * n_used + j] = path(used[i] -> used[j]) for rows
 *   i in [row_begin, row_end).  Diagonal = the raw self-loop edge (:210-217).
 * Error precedence follows the reference: self-loop errors (first used node
 * in order, :211-217) before the unreachable assert (:219).
 * n_threads <= 0 -> 1.  err_a/err_b receive the failing (row, col) indices.
 */
int sgo_shortest_paths(uint32_t n, uint32_t m, const uint32_t* esrc, const uint32_t* edst,
                       const uint64_t* elat, const float* eloss, int directed, const uint32_t* used,
                       uint32_t n_used, uint32_t row_begin, uint32_t row_end, uint64_t* out_lat,
                       float* out_loss, int n_threads, uint32_t* err_a, uint32_t* err_b) {
  if (row_end > n_used || row_begin > row_end) return SGO_ERR_ARG;
  for (uint32_t j = 0; j < n_used; j++)
    if (used[j] >= n) return SGO_ERR_ARG;
  sgo_adj A;
  memset(&A, 0, sizeof(A));
  int rc = adj_build(&A, n, m, esrc, edst, directed);
  if (rc) {
    adj_free(&A);
    return rc;
  }
  sssp_job J;
  memset(&J, 0, sizeof(J));
  J.adj = &A;
  J.elat = elat;
  J.eloss = eloss;
  J.used = used;
  J.n_used = n_used;
  J.out_lat = out_lat;
  J.out_loss = out_loss;
  J.row_begin = row_begin;
  J.row_end = row_end;
  J.next_row = row_begin;
  pthread_mutex_init(&J.mu, NULL);
  if (n_threads <= 1) {
    sssp_worker(&J);
  } else {
    sgo_run_threads(sssp_worker, &J, 0, (uint32_t)n_threads);  /* (a shared job: every thread takes rows) */
  }
  pthread_mutex_destroy(&J.mu);
  if (J.err == SGO_ERR_OOM) {
    adj_free(&A);
    return SGO_ERR_OOM;
  }
  /* self-pair override with the single self-loop (graph/mod.rs:210-217); all
   * used nodes are checked, in order, not just this row block. */
  for (uint32_t j = 0; j < n_used; j++) {
    uint32_t u = used[j], e = 0;
    uint32_t c = count_connecting(&A, u, u, &e);
    if (c != 1) {
      if (err_a) *err_a = j;
      if (err_b) *err_b = j;
      adj_free(&A);
      return c == 0 ? SGO_ERR_NO_EDGE : SGO_ERR_MULTI_EDGE;
    }
    if (j >= row_begin && j < row_end) {
      size_t idx = (size_t)(j - row_begin) * n_used + j;
      out_lat[idx] = elat[e];
      out_loss[idx] = eloss[e];
    }
  }
  adj_free(&A);
  if (J.err == SGO_ERR_UNREACHABLE) {
    if (err_a) *err_a = J.err_row;
    if (err_b) *err_b = J.err_col;
    return SGO_ERR_UNREACHABLE;
  }
  return SGO_OK;
}

/* ------------------------------------------------------------------------- */
/* A whole-table certificate: is a given table compute_shortest_paths' result? */
/* ------------------------------------------------------------------------- */
/* Every edge latency is >= 1 ns (graph/mod.rs:105-107) and the loss fold of
 * graph/mod.rs:322-331 is monotone in the (latency, loss) order of :305-313, so
 * petgraph's Dijkstra (the restatement above) ends with, for every node v != s,
 *     D[s][v] = min over the arcs u -> v of D[s][u] (+) w(u, v),
 * the minimum taken in that order and attained (an arc from a node settled later
 * cannot win: its candidate is later than v's key), with D[s][s] = default().  The
 * solution of these equations is unique: of two solutions, take the node with the
 * smallest value where they differ; its value in one of them comes through a
 * predecessor of strictly smaller latency, where both agree, so the other one
 * reaches it too -- a contradiction.  So a table that satisfies them in every cell
 * (and carries the single self-loop on its diagonal, :210-217) IS the reference's
 * table, bit for bit, with no Dijkstra run: one pass over every in-arc per row,
 * i.e. rows x arcs candidate folds instead of a heap per row.
 * Needs every node used (a path may cross any node: the equations need its value).
 * Returns the number of cells that fail (0: the table is the reference's), the first
 * failing (row, column) in row-major order in bad_row / bad_col, or -SGO_ERR_ARG /
 * -SGO_ERR_OOM.  Rows [row_begin, row_end) of the used order; tab_* hold those rows. */
typedef struct {
  uint32_t n, n_used, row_begin, row_end;
  const uint32_t *in_off, *in_src, *in_edge, *used, *col;
  const uint32_t* in_rec; /* per in-arc {tail, latency (< 2^32), bits(loss)} when every edge latency fits 32 bits */
  const uint64_t* elat;
  const float* eloss;
  const uint64_t* tab_lat;
  const float* tab_loss;
  const uint32_t* self_cnt;  /* self-loops per node */
  const uint32_t* self_edge; /* the first one */
  int64_t next_row;
  int64_t bad;
  uint32_t bad_row, bad_col;
  int err;
  pthread_mutex_t mu;
} fp_job;

static inline uint32_t f32_bits(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return b;
}

static void* fp_worker(void* arg) {
  fp_job* J = (fp_job*)arg;
  const uint32_t n = J->n;
  sgo_pp* D = (sgo_pp*)malloc(((size_t)n + 1) * sizeof(sgo_pp));
  uint64_t* K = (uint64_t*)malloc(((size_t)n + 1) * 8); /* the row as packed keys (the fast path) */
  if (!D || !K) {
    free(D);
    free(K);
    pthread_mutex_lock(&J->mu);
    J->err = SGO_ERR_OOM;
    pthread_mutex_unlock(&J->mu);
    return NULL;
  }
  for (;;) {
    const int64_t row = __atomic_fetch_add(&J->next_row, 1, __ATOMIC_RELAXED);
    if (row >= (int64_t)J->row_end) break;
    const size_t base = (size_t)(row - J->row_begin) * J->n_used;
    const uint32_t s = J->used[row];
    int narrow = J->in_rec != NULL; /* every latency of the row below 2^32: packed keys */
    const uint64_t* tl = J->tab_lat + base;
    const float* tf = J->tab_loss + base;
    uint64_t wide = 0;
    for (uint32_t v = 0; v < n; v++) {
      const uint32_t c = J->col[v];
      wide |= tl[c];
      K[v] = (tl[c] << 32) | f32_bits(tf[c]);
    }
    narrow &= (wide >> 32) == 0;
    if (!narrow)
      for (uint32_t v = 0; v < n; v++) {
        D[v].lat = tl[J->col[v]];
        D[v].loss = tf[J->col[v]];
      }
    const sgo_pp diag = {tl[J->col[s]], tf[J->col[s]]};
    D[s].lat = 0; /* PathProperties::default() at the source */
    D[s].loss = 0.0f;
    K[s] = 0;
    int64_t bad = 0;
    uint32_t first = UINT32_MAX;
    for (uint32_t v = 0; v < n; v++) {
      int ok;
      if (v == s) { /* the diagonal: the single self-loop (graph/mod.rs:210-217) */
        ok = J->self_cnt[v] == 1 && diag.lat == J->elat[J->self_edge[v]] &&
             f32_bits(diag.loss) == f32_bits(J->eloss[J->self_edge[v]]);
      } else if (narrow) {
        /* the same minimum on packed keys: (latency << 32) | bits(loss) orders as (latency, loss)
         * (loss >= 0); a candidate of 2^32 ns or more is later than every key of the row */
        uint64_t best = UINT64_MAX;
        for (uint32_t k = J->in_off[v]; k < J->in_off[v + 1]; k++) {
          const uint32_t* r = J->in_rec + 3 * (size_t)k;
          const uint64_t ku = K[r[0]];
          const uint64_t lat = (ku >> 32) + r[1];
          sgo_pp a = {0, 0.0f};
          float el;
          const uint32_t lb = (uint32_t)ku, eb = r[2];
          memcpy(&a.loss, &lb, 4);
          memcpy(&el, &eb, 4);
          const sgo_pp c = pp_add(a, 0, el);
          const uint64_t kc = lat >> 32 ? UINT64_MAX : (lat << 32) | f32_bits(c.loss);
          best = kc < best ? kc : best;
        }
        ok = best == K[v];
      } else {
        sgo_pp best = {UINT64_MAX, 1.0f};
        int any = 0;
        for (uint32_t k = J->in_off[v]; k < J->in_off[v + 1]; k++) {
          const uint32_t u = J->in_src[k], e = J->in_edge[k];
          if (D[u].lat == UINT64_MAX) continue; /* (a table cell that claims unreachable) */
          const sgo_pp c = pp_add(D[u], J->elat[e], J->eloss[e]);
          if (!any || pp_lt(c, best)) best = c;
          any = 1;
        }
        ok = any && best.lat == D[v].lat && f32_bits(best.loss) == f32_bits(D[v].loss);
      }
      if (!ok) {
        bad++;
        if (J->col[v] < first) first = J->col[v];
      }
    }
    if (bad) {
      pthread_mutex_lock(&J->mu);
      J->bad += bad;
      if ((uint32_t)row < J->bad_row || ((uint32_t)row == J->bad_row && first < J->bad_col)) {
        J->bad_row = (uint32_t)row;
        J->bad_col = first;
      }
      pthread_mutex_unlock(&J->mu);
    }
  }
  free(D);
  free(K);
  return NULL;
}

int64_t sgo_check_fixed_point(uint32_t n, uint32_t m, const uint32_t* esrc, const uint32_t* edst,
                              const uint64_t* elat, const float* eloss, int directed, const uint32_t* used,
                              uint32_t n_used, uint32_t row_begin, uint32_t row_end, const uint64_t* tab_lat,
                              const float* tab_loss, int n_threads, uint32_t* bad_row, uint32_t* bad_col) {
  if (n_used != n || row_begin > row_end || row_end > n_used) return -SGO_ERR_ARG;
  uint32_t* col = (uint32_t*)malloc(((size_t)n + 1) * 4);
  uint32_t* in_off = (uint32_t*)calloc((size_t)n + 1, 4);
  uint32_t* self_cnt = (uint32_t*)calloc((size_t)n + 1, 4);
  uint32_t* self_edge = (uint32_t*)calloc((size_t)n + 1, 4);
  const size_t cap = (directed ? (size_t)m : 2 * (size_t)m) + 1;
  uint32_t* in_src = (uint32_t*)malloc(cap * 4);
  uint32_t* in_edge = (uint32_t*)malloc(cap * 4);
  uint32_t* cur = (uint32_t*)malloc(((size_t)n + 1) * 4);
  int64_t rc = 0;
  if (!col || !in_off || !self_cnt || !self_edge || !in_src || !in_edge || !cur) rc = -SGO_ERR_OOM;
  if (!rc) { /* used must be a permutation of the nodes */
    for (uint32_t v = 0; v < n; v++) col[v] = UINT32_MAX;
    for (uint32_t j = 0; j < n_used && !rc; j++) {
      if (used[j] >= n || col[used[j]] != UINT32_MAX) rc = -SGO_ERR_ARG;
      else col[used[j]] = j;
    }
  }
  if (!rc) { /* in-arcs (self-loops apart: they never win), both directions when undirected */
    for (uint32_t i = 0; i < m; i++) {
      const uint32_t a = esrc[i], b = edst[i];
      if (a >= n || b >= n) {
        rc = -SGO_ERR_ARG;
        break;
      }
      if (a == b) {
        if (self_cnt[a]++ == 0) self_edge[a] = i;
        continue;
      }
      in_off[b + 1]++;
      if (!directed) in_off[a + 1]++;
    }
  }
  if (!rc) {
    for (uint32_t v = 0; v < n; v++) in_off[v + 1] += in_off[v];
    memcpy(cur, in_off, ((size_t)n + 1) * 4);
    for (uint32_t i = 0; i < m; i++) {
      const uint32_t a = esrc[i], b = edst[i];
      if (a == b) continue;
      in_src[cur[b]] = a;
      in_edge[cur[b]++] = i;
      if (!directed) {
        in_src[cur[a]] = b;
        in_edge[cur[a]++] = i;
      }
    }
    /* in-arc records for the packed-key path: tail, latency, loss bits, in CSC order */
    int narrow = 1;
    for (uint32_t i = 0; i < m; i++) narrow &= elat[i] < ((uint64_t)1 << 32);
    uint32_t* rec = narrow ? (uint32_t*)malloc(((size_t)in_off[n] + 1) * 12) : NULL;
    if (rec)
      for (uint32_t k = 0; k < in_off[n]; k++) {
        rec[3 * (size_t)k] = in_src[k];
        rec[3 * (size_t)k + 1] = (uint32_t)elat[in_edge[k]];
        rec[3 * (size_t)k + 2] = f32_bits(eloss[in_edge[k]]);
      }
    fp_job J;
    memset(&J, 0, sizeof(J));
    J.in_rec = rec;
    J.n = n;
    J.n_used = n_used;
    J.row_begin = row_begin;
    J.row_end = row_end;
    J.in_off = in_off;
    J.in_src = in_src;
    J.in_edge = in_edge;
    J.used = used;
    J.col = col;
    J.elat = elat;
    J.eloss = eloss;
    J.tab_lat = tab_lat;
    J.tab_loss = tab_loss;
    J.self_cnt = self_cnt;
    J.self_edge = self_edge;
    J.next_row = row_begin;
    J.bad_row = UINT32_MAX;
    J.bad_col = UINT32_MAX;
    pthread_mutex_init(&J.mu, NULL);
    sgo_run_threads(fp_worker, &J, 0, n_threads < 1 ? 1u : (uint32_t)n_threads);
    pthread_mutex_destroy(&J.mu);
    rc = J.err ? -(int64_t)J.err : J.bad;
    free(rec);
    if (bad_row) *bad_row = J.bad_row;
    if (bad_col) *bad_col = J.bad_col;
  }
  free(col);
  free(in_off);
  free(self_cnt);
  free(self_edge);
  free(in_src);
  free(in_edge);
  free(cur);
  return rc;
}

/*
 * NetworkGraph::get_direct_paths (graph/mod.rs:230-252): the raw edge for every
 * used pair; exactly one edge required; first failing pair in row-major order.
 */
int sgo_direct_paths(uint32_t n, uint32_t m, const uint32_t* esrc, const uint32_t* edst,
                     const uint64_t* elat, const float* eloss, int directed, const uint32_t* used,
                     uint32_t n_used, uint64_t* out_lat, float* out_loss, uint32_t* err_a,
                     uint32_t* err_b) {
  for (uint32_t j = 0; j < n_used; j++)
    if (used[j] >= n) return SGO_ERR_ARG;
  sgo_adj A;
  memset(&A, 0, sizeof(A));
  int rc = adj_build(&A, n, m, esrc, edst, directed);
  if (rc) {
    adj_free(&A);
    return rc;
  }
  uint32_t* cnt = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
  uint32_t* first = (uint32_t*)malloc(((size_t)n + 1) * sizeof(uint32_t));
  if (!cnt || !first) {
    free(cnt);
    free(first);
    adj_free(&A);
    return SGO_ERR_OOM;
  }
  rc = SGO_OK;
  for (uint32_t i = 0; i < n_used && rc == SGO_OK; i++) {
    uint32_t u = used[i];
    for (uint32_t k = A.off[u]; k < A.off[u + 1]; k++) {
      uint32_t v = A.dst[k];
      if (cnt[v]++ == 0) first[v] = A.edge[k];
    }
    for (uint32_t j = 0; j < n_used; j++) {
      uint32_t v = used[j];
      if (cnt[v] != 1) {
        rc = cnt[v] == 0 ? SGO_ERR_NO_EDGE : SGO_ERR_MULTI_EDGE;
        if (err_a) *err_a = i;
        if (err_b) *err_b = j;
        break;
      }
      out_lat[(size_t)i * n_used + j] = elat[first[v]];
      out_loss[(size_t)i * n_used + j] = eloss[first[v]];
    }
    for (uint32_t k = A.off[u]; k < A.off[u + 1]; k++) cnt[A.dst[k]] = 0;
  }
  free(cnt);
  free(first);
  adj_free(&A);
  return rc;
}

/* RoutingInfo::get_smallest_latency_ns (graph/mod.rs:478-480): min over all
 * entries, self pairs included. */
uint64_t sgo_smallest_latency(const uint64_t* lat, size_t count) {
  uint64_t m = UINT64_MAX;
  for (size_t i = 0; i < count; i++)
    if (lat[i] < m) m = lat[i];
  return m;
}

/* ------------------------------------------------------------------------- */
/* RNG: rand_xoshiro 0.7.0 Xoshiro256PlusPlus (host/host.rs:221), seeded by   */
/* SeedableRng::seed_from_u64 = SplitMix64 (sim_config.rs:48-51), and         */
/* rand 0.9.1 StandardUniform f64 = (next_u64 >> 11) * 2^-53 (worker.rs:360). */
/* [external: restated from the published upstream algorithms]               */
/* ------------------------------------------------------------------------- */
static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

uint64_t sgo_splitmix64_next(uint64_t* state) {
  *state += 0x9E3779B97F4A7C15ull;
  uint64_t z = *state;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void sgo_xoshiro_seed_from_u64(uint64_t seed, uint64_t s[4]) {
  uint64_t st = seed;
  for (int i = 0; i < 4; i++) s[i] = sgo_splitmix64_next(&st);
  if (!s[0] && !s[1] && !s[2] && !s[3]) sgo_xoshiro_seed_from_u64(0, s); /* from_seed all-zero guard */
}

uint64_t sgo_xoshiro_next_u64(uint64_t s[4]) {
  uint64_t r = rotl64(s[0] + s[3], 23) + s[0];
  uint64_t t = s[1] << 17;
  s[2] ^= s[0];
  s[3] ^= s[1];
  s[1] ^= s[2];
  s[0] ^= s[3];
  s[2] ^= t;
  s[3] = rotl64(s[3], 45);
  return r;
}

double sgo_xoshiro_next_f64(uint64_t s[4]) {
  return (double)(sgo_xoshiro_next_u64(s) >> 11) * (1.0 / 9007199254740992.0);
}

/* std DefaultHasher = SipHash-1-3 with k0 = k1 = 0 (sim_config.rs:221-225). */
#define SIPROUND                   \
  do {                             \
    v0 += v1;                      \
    v1 = rotl64(v1, 13);           \
    v1 ^= v0;                      \
    v0 = rotl64(v0, 32);           \
    v2 += v3;                      \
    v3 = rotl64(v3, 16);           \
    v3 ^= v2;                      \
    v0 += v3;                      \
    v3 = rotl64(v3, 21);           \
    v3 ^= v0;                      \
    v2 += v1;                      \
    v1 = rotl64(v1, 17);           \
    v1 ^= v2;                      \
    v2 = rotl64(v2, 32);           \
  } while (0)

uint64_t sgo_siphash13(const uint8_t* data, size_t len) {
  uint64_t v0 = 0x736f6d6570736575ull, v1 = 0x646f72616e646f6dull;
  uint64_t v2 = 0x6c7967656e657261ull, v3 = 0x7465646279746573ull;
  size_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t m = 0;
    for (int b = 0; b < 8; b++) m |= (uint64_t)data[i + b] << (8 * b);
    v3 ^= m;
    SIPROUND;
    v0 ^= m;
  }
  uint64_t b = (uint64_t)len << 56;
  for (size_t k = 0; i + k < len; k++) b |= (uint64_t)data[i + k] << (8 * k);
  v3 ^= b;
  SIPROUND;
  v0 ^= b;
  v2 ^= 0xff;
  SIPROUND;
  SIPROUND;
  SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

/* HostInfo.seed (sim_config.rs:50-54,221-225,242): first u64 of the
 * general-seed stream XOR SipHash13(hostname bytes || 0xFF). */
uint64_t sgo_host_seed(uint64_t general_seed, const char* hostname, size_t len) {
  uint64_t s[4];
  sgo_xoshiro_seed_from_u64(general_seed, s);
  uint64_t r = sgo_xoshiro_next_u64(s);
  uint8_t* buf = (uint8_t*)malloc(len + 1);
  memcpy(buf, hostname, len);
  buf[len] = 0xff;
  uint64_t h = sgo_siphash13(buf, len + 1);
  free(buf);
  return r ^ h;
}

/* ------------------------------------------------------------------------- */
/* Worker::send_packet over one round's batch (worker.rs:322-397) + event     */
/* order (event.rs:84-155) + push_packet_to_host (worker.rs:597-607).          */
/* ------------------------------------------------------------------------- */
#define SGO_ST_DELIVERED 0  /* PacketStatus::InetSent, pushed to dst queue */
#define SGO_ST_DROP_LOSS 1  /* InetDropped after the reliability draw (:365-368) */
#define SGO_ST_DROP_NO_DST 2 /* InetDropped, unknown destination, no draw (:341-351) */
#define SGO_ST_SIM_END 3    /* now >= sim_end: returns before anything (:332-335) */

typedef struct {
  uint32_t ip, host;
} ip_host;

static int cmp_ip(const void* a, const void* b) {
  uint32_t x = ((const ip_host*)a)->ip, y = ((const ip_host*)b)->ip;
  return x < y ? -1 : x > y;
}

typedef struct {
  uint64_t t;
  uint32_t src;
  uint64_t eid;
  uint32_t idx;
} ord_item;

/* Event ordering (event.rs:84-155): time, then Packet data by (src_host_id,
 * src_host_event_id).  The key is unique per delivered packet. */
static int cmp_ord(const void* a, const void* b) {
  const ord_item* x = (const ord_item*)a;
  const ord_item* y = (const ord_item*)b;
  if (x->t != y->t) return x->t < y->t ? -1 : 1;
  if (x->src != y->src) return x->src < y->src ? -1 : 1;
  return x->eid < y->eid ? -1 : (x->eid > y->eid);
}

/*
 * Packets appear in each source host's send order (the order send_packet is
 * called for that host); hosts may interleave.  host_row[h] = routing-table row/column of host h's node; the
 * table is n_cols x n_cols (row = source).  rng (4*n_hosts) and event_ctr
 * (n_hosts) are the per-host Xoshiro state and event-id counter, in/out.
 * Outputs: status, deliver_time, event_id per packet; dst_order = delivered
 * packet indices grouped by destination host and ordered as the destination's
 * EventQueue pops them: (time, src_host_id, src_host_event_id); dst_offsets
 * (n_hosts+1); min_deliver = min next-event time (worker.rs:388), min_lat =
 * min used latency (worker.rs:372); UINT64_MAX when nothing was delivered.
 * Returns the number of delivered packets, -1 on a bad argument, or -2 when a
 * delivered packet's send time + latency overflows EmulatedTime (the reference
 * panics).
 * rng_skip (NULL = none): before packet i, its source host's stream takes
 * rng_skip[i] steps for the host's other consumers of Host::random_mut()
 * (host.rs:645-647: getrandom, syscall/handler/random.rs:40; socket port
 * choices, socket.rs:179-858; host_rngDouble / host_rngNextNBytes,
 * host.rs:1288-1300), whatever the packet's status -- the interleaving of those
 * draws with send_packet's own (worker.rs:360) in the host's event order.
 */
int64_t sgo_deliver_round(uint64_t round_end, uint64_t sim_end, uint64_t bootstrap_end,
                          uint32_t n_pkts, const uint32_t* src_host, const uint32_t* dst_ip,
                          const uint32_t* payload_len, const uint64_t* send_time, uint32_t n_hosts,
                          const uint32_t* host_ip, const uint32_t* host_row, uint32_t n_cols,
                          const uint64_t* tab_lat, const float* tab_loss, uint64_t* rng,
                          uint64_t* event_ctr, uint8_t* status, uint64_t* deliver_time,
                          uint64_t* event_id, uint32_t* dst_order, uint32_t* dst_offsets,
                          uint64_t* min_deliver, uint64_t* min_lat, const uint32_t* rng_skip) {
  ip_host* map = (ip_host*)malloc(((size_t)n_hosts + 1) * sizeof(ip_host));
  uint32_t* dst_host = (uint32_t*)malloc(((size_t)n_pkts + 1) * sizeof(uint32_t));
  if (!map || !dst_host) return -1;
  for (uint32_t h = 0; h < n_hosts; h++) {
    map[h].ip = host_ip[h];
    map[h].host = h;
    if (host_row[h] >= n_cols) return -1;
  }
  qsort(map, n_hosts, sizeof(ip_host), cmp_ip);
  uint64_t mind = UINT64_MAX, minl = UINT64_MAX;
  int64_t delivered = 0;
  for (uint32_t i = 0; i < n_pkts; i++) {
    uint32_t s = src_host[i];
    if (s >= n_hosts) return -1;
    uint64_t now = send_time[i];
    deliver_time[i] = 0;
    event_id[i] = UINT64_MAX;
    dst_host[i] = UINT32_MAX;
    if (rng_skip)
      for (uint32_t z = rng_skip[i]; z; z--) (void)sgo_xoshiro_next_u64(&rng[4 * (size_t)s]);
    if (now >= sim_end) {
      status[i] = SGO_ST_SIM_END;
      continue;
    }
    ip_host key = {dst_ip[i], 0};
    ip_host* f = (ip_host*)bsearch(&key, map, n_hosts, sizeof(ip_host), cmp_ip);
    if (!f) {
      status[i] = SGO_ST_DROP_NO_DST;
      continue;
    }
    uint32_t d = f->host;
    size_t cell = (size_t)host_row[s] * n_cols + host_row[d];
    double reliability = (double)(1.0f - tab_loss[cell]); /* worker.rs:357-359,526-531 */
    double chance = sgo_xoshiro_next_f64(&rng[4 * (size_t)s]);
    int bootstrapping = now < bootstrap_end;
    if (!bootstrapping && chance >= reliability && payload_len[i] > 0) {
      status[i] = SGO_ST_DROP_LOSS;
      continue;
    }
    uint64_t delay = tab_lat[cell];
    if (delay < minl) minl = delay;
    uint64_t t = now + delay;
    /* EmulatedTime + SimulationTime: checked_add(..).unwrap() and EMUTIME_MAX = u64::MAX - 1
       (emulated_time.rs:30,98-100,121-126) -- a panic in the reference */
    if (t < now || t == UINT64_MAX) {
      free(map);
      free(dst_host);
      return -2;
    }
    if (t < round_end) t = round_end;
    if (t < mind) mind = t;
    status[i] = SGO_ST_DELIVERED;
    deliver_time[i] = t;
    event_id[i] = event_ctr[s]++;
    dst_host[i] = d;
    delivered++;
  }
  /* bucket by destination, then each bucket in EventQueue pop order. */
  memset(dst_offsets, 0, ((size_t)n_hosts + 1) * sizeof(uint32_t));
  for (uint32_t i = 0; i < n_pkts; i++)
    if (dst_host[i] != UINT32_MAX) dst_offsets[dst_host[i] + 1]++;
  for (uint32_t h = 0; h < n_hosts; h++) dst_offsets[h + 1] += dst_offsets[h];
  ord_item* tmp = (ord_item*)malloc(((size_t)delivered + 1) * sizeof(ord_item));
  uint32_t* cur = (uint32_t*)malloc(((size_t)n_hosts + 1) * sizeof(uint32_t));
  memcpy(cur, dst_offsets, ((size_t)n_hosts + 1) * sizeof(uint32_t));
  for (uint32_t i = 0; i < n_pkts; i++)
    if (dst_host[i] != UINT32_MAX) {
      ord_item it = {deliver_time[i], src_host[i], event_id[i], i};
      tmp[cur[dst_host[i]]++] = it;
    }
  for (uint32_t h = 0; h < n_hosts; h++) {
    uint32_t b = dst_offsets[h], e = dst_offsets[h + 1];
    qsort(tmp + b, e - b, sizeof(ord_item), cmp_ord);
  }
  for (int64_t k = 0; k < delivered; k++) dst_order[k] = tmp[k].idx;
  free(tmp);
  free(cur);
  free(map);
  free(dst_host);
  *min_deliver = mind;
  *min_lat = minl;
  return delivered;
}

/* ------------------------------------------------------------------------- */
/* Router inbound CoDel queue (router/codel_queue.rs), one queue per host    */
/* ------------------------------------------------------------------------- */
/* State per host (SoA, the same layout as the HIP side):
 *   flags  bit0 mode == Drop, bit1 interval_end is Some, bit2 drop_next is Some
 *   interval_end, drop_next (EmulatedTime ns), cur/prev drop counts, bytes
 *   (total_bytes_stored), and the FIFO as a ring of `cap` slots per host:
 *   head/tail are running counters, slot = h * cap + (counter % cap).
 * Events are grouped by ascending host, each host's in its order:
 *   kind 0 = push(packet, len, now)   (codel_queue.rs:303-317)
 *   kind 1 = pop(now) -> packet|None  (codel_queue.rs:125-148)
 * pop_result[e] = the popped packet or UINT32_MAX; pkt_status[packet] = 1 when
 * it leaves through a pop, 2 when CoDel drops it (RouterDropped). */
#define CD_TARGET 10000000ull     /* codel_queue.rs:23  10 ms */
#define CD_INTERVAL 100000000ull  /* codel_queue.rs:28 100 ms */
#define CD_MTU 1500ull            /* definitions.h:124 CONFIG_MTU */
#define EMU_MAX (UINT64_MAX - 1)  /* emulated_time.rs:30 EMUTIME_MAX */
enum { CD_DROP = 1, CD_HAS_IEND = 2, CD_HAS_DNEXT = 4 };

typedef struct {
  uint8_t flags;
  uint64_t iend, dnext, cur, prev, bytes;
  uint32_t head, tail;
  uint32_t* rpkt;
  uint64_t* rts;
  uint32_t* rlen;
  uint32_t cap;
  uint8_t* status;
  uint32_t n_status;
  int err;
} cd_q;

static uint64_t cd_sat_add(uint64_t t, uint64_t d) {  /* EmulatedTime::saturating_add */
  return (t > EMU_MAX - d) ? EMU_MAX : t + d;
}
static uint64_t cd_since(uint64_t now, uint64_t t) { return now > t ? now - t : 0; }

/* apply_control_law (codel_queue.rs:285-298): time + round(INTERVAL / sqrt(count)) */
uint64_t sgo_codel_control_law(uint64_t t, uint64_t count) {
  const double interval = (double)CD_INTERVAL;
  const double s = count == 0 ? 1.0 : sqrt((double)count);
  const double div = interval / s;
  const uint64_t inc = (uint64_t)round(div);
  return cd_sat_add(t, inc);
}

static void cd_drop(cd_q* q, uint32_t pkt) {
  if (pkt < q->n_status) q->status[pkt] = 2;
  else q->err = -3;
}

/* process_standing_delay (:231-262) */
static int cd_standing(cd_q* q, uint64_t now, uint64_t sd) {
  if (sd < CD_TARGET || q->bytes <= CD_MTU) {
    q->flags &= (uint8_t)~CD_HAS_IEND;
    return 0;
  }
  if (q->flags & CD_HAS_IEND) return now >= q->iend;
  q->iend = cd_sat_add(now, CD_INTERVAL);
  q->flags |= CD_HAS_IEND;
  return 0;
}

/* codel_pop / dodequeue (:204-227): 1 = got (pkt, ok) */
static int cd_pop_front(cd_q* q, uint64_t now, uint32_t* pkt, int* ok) {
  if (q->head == q->tail) {
    q->flags &= (uint8_t)~CD_HAS_IEND;
    return 0;
  }
  const uint32_t slot = q->head % q->cap;
  q->head++;
  *pkt = q->rpkt[slot];
  const uint64_t len = q->rlen[slot];
  q->bytes = q->bytes > len ? q->bytes - len : 0;
  *ok = cd_standing(q, now, cd_since(now, q->rts[slot]));
  return 1;
}

static int cd_should_drop(const cd_q* q, uint64_t now) { return (q->flags & CD_HAS_DNEXT) && now >= q->dnext; }
static int cd_dropping_recently(const cd_q* q, uint64_t now) {
  return (q->flags & CD_HAS_DNEXT) && cd_since(now, q->dnext) < 16 * CD_INTERVAL;
}

/* pop (:125-148) with drop_from_store_mode (:150-170) and drop_from_drop_mode (:172-201) */
static uint32_t cd_pop(cd_q* q, uint64_t now) {
  uint32_t pkt;
  int ok;
  if (!cd_pop_front(q, now, &pkt, &ok)) {
    q->flags &= (uint8_t)~CD_DROP;
    return UINT32_MAX;
  }
  if (!ok) {
    q->flags &= (uint8_t)~CD_DROP;
    return pkt;
  }
  if (!(q->flags & CD_DROP)) {  /* drop_from_store_mode */
    cd_drop(q, pkt);
    uint32_t nxt;
    int nok;
    const int has = cd_pop_front(q, now, &nxt, &nok);
    q->flags |= CD_DROP;
    const uint64_t delta = q->cur > q->prev ? q->cur - q->prev : 0;
    q->cur = (cd_dropping_recently(q, now) && delta > 1) ? delta : 1;
    q->dnext = sgo_codel_control_law(now, q->cur);
    q->flags |= CD_HAS_DNEXT;
    q->prev = q->cur;
    return has ? nxt : UINT32_MAX;
  }
  /* drop_from_drop_mode */
  int has = 1;
  while (has && (q->flags & CD_DROP) && cd_should_drop(q, now)) {
    cd_drop(q, pkt);
    q->cur++;
    has = cd_pop_front(q, now, &pkt, &ok);
    if (has && ok)
      q->dnext = sgo_codel_control_law(q->dnext, q->cur);
    else
      q->flags &= (uint8_t)~CD_DROP;
  }
  return has ? pkt : UINT32_MAX;
}

/* Hosts h = phase, phase + stride, ...; off (n_hosts + 1, or NULL: one pass over every host in
 * order) gives each host's first event -- the multi-threaded CPU baselines (sgo_*_run_mt) run one
 * thread per phase, hosts round-robin over the threads as thread_per_core.rs:62-64 deals them. */
static int codel_impl(uint32_t n_hosts, uint32_t cap, uint8_t* flags, uint64_t* iend, uint64_t* dnext,
                      uint64_t* cur, uint64_t* prev, uint64_t* bytes, uint32_t* head, uint32_t* tail,
                      uint32_t* ring_pkt, uint64_t* ring_ts, uint32_t* ring_len, uint32_t n_events,
                      const uint32_t* host, const uint8_t* kind, const uint64_t* time, const uint32_t* pkt,
                      const uint32_t* len, uint32_t* pop_result, uint8_t* pkt_status, uint32_t n_status,
                      const uint32_t* off, uint32_t stride, uint32_t phase) {
  if (!cap) return -1;
  uint32_t e = 0;
  for (uint32_t h = phase; h < n_hosts; h += stride) {
    if (off) e = off[h];
    cd_q q = {flags[h], iend[h], dnext[h], cur[h], prev[h], bytes[h], head[h], tail[h],
              ring_pkt + (size_t)h * cap, ring_ts + (size_t)h * cap, ring_len + (size_t)h * cap, cap,
              pkt_status, n_status, 0};
    for (; e < n_events && host[e] == h; e++) {
      pop_result[e] = UINT32_MAX;
      if (kind[e] == 0) {
        if (q.tail - q.head >= cap) return -2;  /* the caller's ring is too small (the reference has no limit) */
        const uint32_t slot = q.tail % cap;
        q.rpkt[slot] = pkt[e];
        q.rts[slot] = time[e];
        q.rlen[slot] = len[e];
        q.tail++;
        q.bytes += len[e];
      } else {
        const uint32_t p = cd_pop(&q, time[e]);
        pop_result[e] = p;
        if (p != UINT32_MAX) {
          if (p < n_status) pkt_status[p] = 1;
          else return -3;
        }
      }
      if (q.err) return q.err;
    }
    flags[h] = q.flags;
    iend[h] = q.iend;
    dnext[h] = q.dnext;
    cur[h] = q.cur;
    prev[h] = q.prev;
    bytes[h] = q.bytes;
    head[h] = q.head;
    tail[h] = q.tail;
  }
  return off || e == n_events ? 0 : -4;  /* -4: events not grouped by ascending host (or host >= n_hosts) */
}

int sgo_codel_run(uint32_t n_hosts, uint32_t cap, uint8_t* flags, uint64_t* iend, uint64_t* dnext,
                  uint64_t* cur, uint64_t* prev, uint64_t* bytes, uint32_t* head, uint32_t* tail,
                  uint32_t* ring_pkt, uint64_t* ring_ts, uint32_t* ring_len, uint32_t n_events,
                  const uint32_t* host, const uint8_t* kind, const uint64_t* time, const uint32_t* pkt,
                  const uint32_t* len, uint32_t* pop_result, uint8_t* pkt_status, uint32_t n_status) {
  return codel_impl(n_hosts, cap, flags, iend, dnext, cur, prev, bytes, head, tail, ring_pkt, ring_ts, ring_len,
                    n_events, host, kind, time, pkt, len, pop_result, pkt_status, n_status, NULL, 1, 0);
}

/* ------------------------------------------------------------------------- */
/* Inbound pipeline: router CoDel queue -> relay_inet_in (token bucket)      */
/* ------------------------------------------------------------------------- */
/* Per host, over a window of simulated time (relay/mod.rs, relay/token_bucket.rs,
 * host.rs:781-786 and :903-924):
 *   a Packet event at t (the delivery's arrival, EventQueue order) pushes the
 *   packet into the router's CoDel queue and notifies relay_inet_in; an Idle
 *   relay schedules its forward task at t (a Local event: after every Packet
 *   event at t, event.rs:103-112; it takes an event id, host.rs:649-653);
 *   the task pops the queue until it is empty or the token bucket blocks, and
 *   then reschedules itself after the conforming duration.
 * Relay state per host: rflags bit0 Pending, bit1 the pending task was never
 * queued (at or after sim_end, host.rs:703-709), bit2 a cached packet
 * (RelayCached); task_time, cached packet/len; token bucket capacity, balance,
 * refill increment, last refill (1 ms interval, token_bucket.rs:20-60,
 * relay/mod.rs:296-309).
 * fwd_time[packet] = the time the relay pushed it to the interface
 * (RelayForwarded) -- status 1 -- or status 2 when CoDel dropped it. */
#define TB_INTERVAL 1000000ull /* relay/mod.rs:297 refill every 1 ms */
enum { RL_PENDING = 1, RL_NEVER = 2, RL_CACHED = 4 };

typedef struct {
  uint64_t cap, bal, inc, last, interval;
} tb_t;

/* lazy_refill (token_bucket.rs:124-158): returns the span to the next refill */
static uint64_t tb_lazy_refill(tb_t* b, uint64_t now) {
  uint64_t span = now - b->last; /* duration_since: now >= last_refill */
  if (span >= b->interval) {
    const uint64_t n = span / b->interval;
    const uint64_t tokens = (b->inc != 0 && n > UINT64_MAX / b->inc) ? UINT64_MAX : b->inc * n;
    uint64_t bal = (b->bal > UINT64_MAX - tokens) ? UINT64_MAX : b->bal + tokens;
    b->bal = bal > b->cap ? b->cap : bal;
    const uint64_t inc = (n > UINT64_MAX / b->interval) ? UINT64_MAX : b->interval * n;
    b->last = cd_sat_add(b->last, inc);
    span = now - b->last;
  }
  return b->interval - span;
}

/* conforming_remove (token_bucket.rs:76-86): 1 and balance -= dec, or 0 and *wait */
static int tb_remove(tb_t* b, uint64_t dec, uint64_t now, uint64_t* wait) {
  const uint64_t next = tb_lazy_refill(b, now);
  if (b->bal >= dec) {
    b->bal -= dec;
    return 1;
  }
  const uint64_t need = dec > b->bal ? dec - b->bal : 0; /* compute_conforming_duration (:93-118) */
  const uint64_t nref = need / b->inc + (need % b->inc ? 1 : 0);
  if (nref == 0) *wait = 0;
  else if (nref == 1) *wait = next;
  else {
    const uint64_t m = nref - 1;
    const uint64_t extra = (m > UINT64_MAX / b->interval) ? UINT64_MAX : b->interval * m;
    *wait = next > UINT64_MAX - extra ? UINT64_MAX : next + extra;
  }
  return 0;
}

static int inbound_impl(uint32_t n_hosts, uint32_t cap, uint8_t* flags, uint64_t* iend, uint64_t* dnext,
                        uint64_t* cur, uint64_t* prev, uint64_t* bytes, uint32_t* head, uint32_t* tail,
                        uint32_t* ring_pkt, uint64_t* ring_ts, uint32_t* ring_len, uint8_t* rflags,
                        uint64_t* task_time, uint64_t* task_id, uint64_t* task_born, uint32_t* cached_pkt,
                        uint32_t* cached_len, uint64_t* tb_cap, uint64_t* tb_bal, uint64_t* tb_inc, uint64_t* tb_last,
                        uint32_t n_arr, const uint32_t* host, const uint64_t* time, const uint32_t* pkt,
                        const uint32_t* len, uint64_t window_end, uint64_t bootstrap_end, uint64_t sim_end,
                        uint64_t* event_ctr, uint64_t* fwd_time, uint8_t* pkt_status, uint32_t n_status,
                        const uint32_t* off, uint32_t stride, uint32_t phase) {
  if (!cap) return -1;
  uint32_t e = 0;
  for (uint32_t h = phase; h < n_hosts; h += stride) {
    if (off) e = off[h];
    cd_q q = {flags[h], iend[h], dnext[h], cur[h], prev[h], bytes[h], head[h], tail[h],
              ring_pkt + (size_t)h * cap, ring_ts + (size_t)h * cap, ring_len + (size_t)h * cap, cap,
              pkt_status, n_status, 0};
    tb_t tb = {tb_cap[h], tb_bal[h], tb_inc[h], tb_last[h], TB_INTERVAL};
    uint8_t rf = rflags[h];
    uint64_t tt = task_time[h], tid = task_id[h], tborn = task_born[h];
    uint32_t cp = cached_pkt[h], cl = cached_len[h];
    uint32_t e1 = e;
    while (e1 < n_arr && host[e1] == h) e1++;
    for (;;) {
      const int has_arr = e < e1;
      const int has_task = (rf & RL_PENDING) && !(rf & RL_NEVER) && tt < window_end;
      if (has_arr && time[e] >= window_end) return -5; /* arrivals must precede the window end */
      if (has_arr && (!has_task || time[e] <= tt)) { /* Packet event (before a Local one at equal time) */
        const uint64_t now = time[e];
        if (q.tail - q.head >= cap) return -2;
        const uint32_t slot = q.tail % cap;
        q.rpkt[slot] = pkt[e];
        q.rts[slot] = now;
        q.rlen[slot] = len[e];
        q.tail++;
        q.bytes += len[e];
        if (!(rf & RL_PENDING)) { /* notify: Idle -> forward_later(ZERO), a Local event (host.rs:690-697) */
          tid = event_ctr[h]++;
          tborn = now;
          rf |= RL_PENDING;
          if (now >= sim_end) rf |= RL_NEVER;
          tt = now;
        }
        e++;
      } else if (has_task) { /* the relay's forward task at tt */
        const uint64_t now = tt;
        rf &= (uint8_t)~RL_PENDING; /* run_forward_task: Idle, then forward_now */
        for (;;) {
          uint32_t p, l;
          if (rf & RL_CACHED) {
            p = cp;
            l = cl;
            rf &= (uint8_t)~RL_CACHED;
          } else {
            const uint32_t popped = cd_pop(&q, now);
            if (q.err) return q.err;
            if (popped == UINT32_MAX) break; /* queue empty: Idle */
            p = popped;
            const uint32_t slot = (q.head - 1) % cap; /* the popped element's length */
            l = q.rlen[slot];
          }
          uint64_t wait;
          if (now >= bootstrap_end && !tb_remove(&tb, l, now, &wait)) {
            rf |= RL_CACHED; /* RelayCached; forward_later(wait) */
            cp = p;
            cl = l;
            tid = event_ctr[h]++;
            tborn = now;
            rf |= RL_PENDING;
            const uint64_t at = now > UINT64_MAX - wait ? UINT64_MAX : now + wait;
            if (at >= sim_end) rf |= RL_NEVER;
            tt = at;
            break;
          }
          if (p < n_status) {
            pkt_status[p] = 1; /* RelayForwarded -> the interface */
            fwd_time[p] = now;
          } else {
            return -3;
          }
        }
      } else {
        break;
      }
    }
    if (e != e1) return -4;
    flags[h] = q.flags;
    iend[h] = q.iend;
    dnext[h] = q.dnext;
    cur[h] = q.cur;
    prev[h] = q.prev;
    bytes[h] = q.bytes;
    head[h] = q.head;
    tail[h] = q.tail;
    rflags[h] = rf;
    task_time[h] = tt;
    task_id[h] = tid;
    task_born[h] = tborn;
    cached_pkt[h] = cp;
    cached_len[h] = cl;
    tb_bal[h] = tb.bal;
    tb_last[h] = tb.last;
  }
  return off || e == n_arr ? 0 : -4;
}

int sgo_inbound_run(uint32_t n_hosts, uint32_t cap, uint8_t* flags, uint64_t* iend, uint64_t* dnext,
                    uint64_t* cur, uint64_t* prev, uint64_t* bytes, uint32_t* head, uint32_t* tail,
                    uint32_t* ring_pkt, uint64_t* ring_ts, uint32_t* ring_len, uint8_t* rflags, uint64_t* task_time,
                    uint64_t* task_id, uint64_t* task_born, uint32_t* cached_pkt, uint32_t* cached_len, uint64_t* tb_cap, uint64_t* tb_bal,
                    uint64_t* tb_inc, uint64_t* tb_last, uint32_t n_arr, const uint32_t* host,
                    const uint64_t* time, const uint32_t* pkt, const uint32_t* len, uint64_t window_end,
                    uint64_t bootstrap_end, uint64_t sim_end, uint64_t* event_ctr, uint64_t* fwd_time,
                    uint8_t* pkt_status, uint32_t n_status) {
  return inbound_impl(n_hosts, cap, flags, iend, dnext, cur, prev, bytes, head, tail, ring_pkt, ring_ts, ring_len,
                      rflags, task_time, task_id, task_born, cached_pkt, cached_len, tb_cap, tb_bal, tb_inc, tb_last,
                      n_arr, host, time, pkt, len, window_end, bootstrap_end, sim_end, event_ctr, fwd_time,
                      pkt_status, n_status, NULL, 1, 0);
}

/* Outbound pipeline: NetworkInterface (fifo qdisc) -> relay_inet_out -> Router
 * -> Worker::send_packet, per host over a window (relay/mod.rs:111-275,
 * host.rs:930-945, interface.rs:168-260, router/mod.rs:41-43).  A host's sends
 * are one FIFO in priority (= creation) order; the relay pops and forwards
 * while its token bucket allows, a packet to the host's own address goes back
 * to the interface without tokens, any other is sent at the task's time.  The
 * FIFO is held as a ring of `cap` slots {packet, len, dst, payload_len}; the
 * packet the relay caches (next_packet) is the slot at head - 1, and a call's
 * pushes may not reach the oldest slot it still needs (the library's bound,
 * -2 here).  Same-time order (event.rs:84-155): a send made by a Packet
 * event (ev_id UINT64_MAX), or with no keys (ev_id NULL), precedes a forward
 * task at its time; a send made by a Local event follows a task at its time
 * iff the task was created first: (task created, task id) < (ev_born, ev_id).
 * Task ids come from event_ctr (host.rs:649-653), creation times are the
 * times forward_later ran (relay/mod.rs:145-157, host.rs:690-697).  A
 * Local send's id moves event_ctr past it (the event exists, so the host's
 * counter is beyond its id): tasks the send schedules are numbered after it.
 * Sent packets are appended to out_* (send_packet order: hosts ascending).
 * Returns 0, or -2 ring full, -3 packet id >= n_status, -4 not grouped,
 * -5 a send at or after window_end, -6 a host's send times decrease,
 * -7 more than out_cap sent. */
/* out_* [out_begin, out_end): this pass's output slots; *n_out: the slots it used (from out_begin) */
static int outbound_impl(uint32_t n_hosts, uint32_t cap, const uint32_t* host_ip, uint32_t* head, uint32_t* tail,
                         uint32_t* ring_pkt, uint32_t* ring_len, uint32_t* ring_dst, uint32_t* ring_pay,
                         uint8_t* rflags, uint64_t* task_time, uint64_t* task_id, uint64_t* task_born, uint64_t* tb_cap,
                         uint64_t* tb_bal, uint64_t* tb_inc, uint64_t* tb_last, uint32_t n_sends, const uint32_t* host,
                         const uint64_t* time, const uint32_t* pkt, const uint32_t* len, const uint32_t* pay,
                         const uint32_t* dst, const uint64_t* ev_id, const uint64_t* ev_born, uint64_t window_end,
                         uint64_t bootstrap_end, uint64_t sim_end, uint64_t* event_ctr, uint64_t* fwd_time,
                         uint8_t* pkt_status, uint32_t n_status, uint32_t* out_host, uint32_t* out_dst,
                         uint32_t* out_pay, uint64_t* out_time, uint32_t* out_pkt, uint32_t out_begin,
                         uint32_t out_end, uint32_t* n_out, const uint32_t* off, uint32_t stride, uint32_t phase) {
  if (!cap) return -1;
  if ((ev_id == NULL) != (ev_born == NULL)) return -1;
  uint32_t e = 0, no = out_begin;
  const uint32_t out_cap = out_end;
  *n_out = 0;
  for (uint32_t h = phase; h < n_hosts; h += stride) {
    if (off) e = off[h];
    const size_t base = (size_t)h * cap;
    tb_t tb = {tb_cap[h], tb_bal[h], tb_inc[h], tb_last[h], TB_INTERVAL};
    uint8_t rf = rflags[h];
    uint64_t tt = task_time[h], tid = task_id[h], tborn = task_born[h];
    uint32_t hd = head[h], tl = tail[h];
    const uint32_t oldest = hd - ((rf & RL_CACHED) ? 1u : 0u);
    uint32_t e1 = e;
    const uint32_t e_first = e;
    while (e1 < n_sends && host[e1] == h) e1++;
    uint64_t last = 0;
    for (;;) {
      const int has_send = e < e1;
      const int has_task = (rf & RL_PENDING) && !(rf & RL_NEVER) && tt < window_end;
      if (has_send && time[e] >= window_end) return -5;
      if (has_send && time[e] < last) return -6;
      if (has_send && ev_id && e > e_first && time[e] == time[e - 1]) { /* execution order within a time */
        const int pk = ev_id[e] == UINT64_MAX, ppk = ev_id[e - 1] == UINT64_MAX;
        if ((pk && !ppk) || (!pk && !ppk && (ev_born[e] < ev_born[e - 1] ||
                                             (ev_born[e] == ev_born[e - 1] && ev_id[e] < ev_id[e - 1]))))
          return -6;
      }
      int send_first = has_send && (!has_task || time[e] < tt);
      if (has_send && has_task && time[e] == tt) {
        /* one EmulatedTime: Packet events, then Local events by id = creation order */
        if (ev_id && ev_id[e] != UINT64_MAX && ev_born[e] == tborn && ev_id[e] == tid)
          return -6; /* the send's key is the pending task's: two events with one id */
        send_first = !ev_id || ev_id[e] == UINT64_MAX || ev_born[e] < tborn ||
                     (ev_born[e] == tborn && ev_id[e] < tid);
      }
      if (send_first) { /* add_data_source + Relay::notify */
        const uint64_t now = time[e];
        last = now;
        /* the sending event exists: the counter is past its id (a no-op for ids from this counter) */
        if (ev_id && ev_id[e] != UINT64_MAX && event_ctr[h] <= ev_id[e]) event_ctr[h] = ev_id[e] + 1;
        if (tl - oldest >= cap) return -2;
        const size_t slot = base + tl % cap;
        ring_pkt[slot] = pkt[e];
        ring_len[slot] = len[e];
        ring_dst[slot] = dst[e];
        ring_pay[slot] = pay[e];
        tl++;
        if (!(rf & RL_PENDING)) { /* Idle -> forward_later(ZERO) */
          tid = event_ctr[h]++;
          tborn = now;
          rf |= RL_PENDING;
          if (now >= sim_end) rf |= RL_NEVER;
          tt = now;
        }
        e++;
      } else if (has_task) { /* run_forward_task -> forward_until_blocked */
        const uint64_t now = tt;
        /* the next send's event exists from its creation on: a task running after that time
           (it may reschedule itself) finds the host's counter past its id.  At the creation
           time itself the order of the task and the creating event is not known: no bump */
        if (has_send && ev_id && ev_id[e] != UINT64_MAX && tt > ev_born[e] && event_ctr[h] <= ev_id[e])
          event_ctr[h] = ev_id[e] + 1;
        rf &= (uint8_t)~RL_PENDING;
        for (;;) {
          size_t slot;
          if (rf & RL_CACHED) { /* next_packet.take() */
            slot = base + (hd - 1) % cap;
            rf &= (uint8_t)~RL_CACHED;
          } else {
            if (hd == tl) break; /* the interface is empty: Idle */
            slot = base + hd % cap;
            hd++;
          }
          const uint32_t p = ring_pkt[slot];
          const int local = ring_dst[slot] == host_ip[h]; /* relay/mod.rs:222-226 */
          uint64_t wait;
          if (!local && now >= bootstrap_end && !tb_remove(&tb, ring_len[slot], now, &wait)) {
            rf |= RL_CACHED | RL_PENDING; /* RelayCached; forward_later(wait) */
            tid = event_ctr[h]++;
            tborn = now;
            const uint64_t at = now > UINT64_MAX - wait ? UINT64_MAX : now + wait;
            if (at >= sim_end) rf |= RL_NEVER;
            tt = at;
            break;
          }
          if (p >= n_status) return -3;
          pkt_status[p] = local ? 2 : 1;
          fwd_time[p] = now;
          if (!local) { /* Router::push -> Worker::send_packet(now) */
            if (no >= out_cap) return -7;
            out_host[no] = h;
            out_dst[no] = ring_dst[slot];
            out_pay[no] = ring_pay[slot];
            out_time[no] = now;
            out_pkt[no] = p;
            no++;
          }
        }
      } else {
        break;
      }
    }
    if (e != e1) return -4;
    head[h] = hd;
    tail[h] = tl;
    rflags[h] = rf;
    task_time[h] = tt;
    task_id[h] = tid;
    task_born[h] = tborn;
    tb_bal[h] = tb.bal;
    tb_last[h] = tb.last;
  }
  *n_out = no - out_begin;
  return off || e == n_sends ? 0 : -4;
}

int sgo_outbound_run(uint32_t n_hosts, uint32_t cap, const uint32_t* host_ip, uint32_t* head, uint32_t* tail,
                     uint32_t* ring_pkt, uint32_t* ring_len, uint32_t* ring_dst, uint32_t* ring_pay,
                     uint8_t* rflags, uint64_t* task_time, uint64_t* task_id, uint64_t* task_born, uint64_t* tb_cap,
                     uint64_t* tb_bal, uint64_t* tb_inc, uint64_t* tb_last, uint32_t n_sends, const uint32_t* host,
                     const uint64_t* time, const uint32_t* pkt, const uint32_t* len, const uint32_t* pay,
                     const uint32_t* dst, const uint64_t* ev_id, const uint64_t* ev_born, uint64_t window_end, uint64_t bootstrap_end, uint64_t sim_end, uint64_t* event_ctr,
                     uint64_t* fwd_time, uint8_t* pkt_status, uint32_t n_status, uint32_t* out_host,
                     uint32_t* out_dst, uint32_t* out_pay, uint64_t* out_time, uint32_t* out_pkt, uint32_t out_cap,
                     uint32_t* n_out) {
  return outbound_impl(n_hosts, cap, host_ip, head, tail, ring_pkt, ring_len, ring_dst, ring_pay, rflags, task_time,
                       task_id, task_born, tb_cap, tb_bal, tb_inc, tb_last, n_sends, host, time, pkt, len, pay, dst,
                       ev_id, ev_born, window_end, bootstrap_end, sim_end, event_ctr, fwd_time, pkt_status, n_status,
                       out_host, out_dst, out_pay, out_time, out_pkt, 0, out_cap, n_out, NULL, 1, 0);
}

/* Test hook: TokenBucket::conforming_remove_inner on an explicit state
 * {capacity, balance, refill_increment, last_refill, refill_interval}.
 * Returns 1 (ok, balance updated) or 0 (*wait = conforming duration). */
int sgo_token_bucket_remove(uint64_t* st, uint64_t dec, uint64_t now, uint64_t* wait) {
  tb_t b = {st[0], st[1], st[2], st[3], st[4]};
  const int ok = tb_remove(&b, dec, now, wait);
  st[1] = b.bal;
  st[3] = b.last;
  return ok;
}

/* ------------------------------------------------------------------------- */
/* Multi-threaded deliver_round: the CPU baseline on the host's cores.       */
/* ------------------------------------------------------------------------- */
/* The reference runs Worker::send_packet on N worker threads, hosts
 * round-robin to threads (thread_per_core.rs:62-64), each destination queue
 * behind a lock.  This restatement gives each thread a contiguous range of
 * source hosts (a host's packets stay on one thread: its RNG stream is
 * sequential), then buckets by destination with per-thread histograms and a
 * parallel per-destination sort.  Results are identical to sgo_deliver_round
 * (per-host streams are independent; the bucket order is a total order). */
typedef struct {
  /* inputs */
  uint64_t round_end, sim_end, bootstrap_end;
  const uint32_t *src_host, *dst_ip, *payload_len;
  const uint64_t* send_time;
  uint32_t n_hosts, n_cols;
  const uint32_t* host_row;
  const uint64_t* tab_lat;
  const float* tab_loss;
  const ip_host* map;
  uint64_t *rng, *event_ctr;
  /* outputs */
  uint8_t* status;
  uint64_t *deliver_time, *event_id;
  uint32_t* dst_host;
  uint32_t *dst_offsets, *dst_order;
  ord_item* tmp;
  /* partition */
  uint32_t T;
  const uint32_t* pkt_begin; /* T + 1 packet boundaries (host-aligned) */
  uint32_t* hist;            /* T x (n_hosts + 1) */
  uint64_t *mind, *minl;
  int64_t* delivered;
  int err;
} mt_job;

typedef struct {
  mt_job* J;
  uint32_t t;
  int phase;
} mt_arg;

static void* mt_worker(void* p) {
  mt_arg* A = (mt_arg*)p;
  mt_job* J = A->J;
  const uint32_t t = A->t, H = J->n_hosts;
  if (A->phase == 0) { /* send_packet for this thread's hosts, then its destination histogram */
    uint64_t mind = UINT64_MAX, minl = UINT64_MAX;
    int64_t nd = 0;
    uint32_t* hist = J->hist + (size_t)t * (H + 1);
    for (uint32_t i = J->pkt_begin[t]; i < J->pkt_begin[t + 1]; i++) {
      const uint32_t s = J->src_host[i];
      const uint64_t now = J->send_time[i];
      J->deliver_time[i] = 0;
      J->event_id[i] = UINT64_MAX;
      J->dst_host[i] = UINT32_MAX;
      if (now >= J->sim_end) {
        J->status[i] = SGO_ST_SIM_END;
        continue;
      }
      ip_host key = {J->dst_ip[i], 0};
      const ip_host* f = (const ip_host*)bsearch(&key, J->map, H, sizeof(ip_host), cmp_ip);
      if (!f) {
        J->status[i] = SGO_ST_DROP_NO_DST;
        continue;
      }
      const uint32_t d = f->host;
      const size_t cell = (size_t)J->host_row[s] * J->n_cols + J->host_row[d];
      const double reliability = (double)(1.0f - J->tab_loss[cell]);
      const double chance = sgo_xoshiro_next_f64(&J->rng[4 * (size_t)s]);
      if (!(now < J->bootstrap_end) && chance >= reliability && J->payload_len[i] > 0) {
        J->status[i] = SGO_ST_DROP_LOSS;
        continue;
      }
      const uint64_t delay = J->tab_lat[cell];
      if (delay < minl) minl = delay;
      uint64_t tt = now + delay;
      if (tt < now || tt == UINT64_MAX) { /* EmulatedTime overflow: a panic in the reference */
        J->err = 1;
        tt = UINT64_MAX - 1;
      }
      if (tt < J->round_end) tt = J->round_end;
      if (tt < mind) mind = tt;
      J->status[i] = SGO_ST_DELIVERED;
      J->deliver_time[i] = tt;
      J->event_id[i] = J->event_ctr[s]++;
      J->dst_host[i] = d;
      hist[d]++;
      nd++;
    }
    J->mind[t] = mind;
    J->minl[t] = minl;
    J->delivered[t] = nd;
  } else if (A->phase == 1) { /* scatter this thread's packets to their destination slots */
    uint32_t* cur = J->hist + (size_t)t * (H + 1); /* now: this thread's start in each bucket */
    for (uint32_t i = J->pkt_begin[t]; i < J->pkt_begin[t + 1]; i++) {
      const uint32_t d = J->dst_host[i];
      if (d == UINT32_MAX) continue;
      ord_item it = {J->deliver_time[i], J->src_host[i], J->event_id[i], i};
      J->tmp[cur[d]++] = it;
    }
  } else { /* sort destination buckets [t*H/T, (t+1)*H/T) */
    const uint32_t h0 = (uint32_t)((uint64_t)H * t / J->T), h1 = (uint32_t)((uint64_t)H * (t + 1) / J->T);
    for (uint32_t h = h0; h < h1; h++) {
      const uint32_t b = J->dst_offsets[h], e = J->dst_offsets[h + 1];
      qsort(J->tmp + b, e - b, sizeof(ord_item), cmp_ord);
      for (uint32_t k = b; k < e; k++) J->dst_order[k] = J->tmp[k].idx;
    }
  }
  return NULL;
}

static void mt_run(mt_job* J, int phase) {
  mt_arg args[64];
  for (uint32_t t = 0; t < J->T; t++) args[t] = (mt_arg){J, t, phase};
  sgo_run_threads(mt_worker, args, sizeof(mt_arg), J->T);
}

int64_t sgo_deliver_round_mt(uint64_t round_end, uint64_t sim_end, uint64_t bootstrap_end, uint32_t n_pkts,
                             const uint32_t* src_host, const uint32_t* dst_ip, const uint32_t* payload_len,
                             const uint64_t* send_time, uint32_t n_hosts, const uint32_t* host_ip,
                             const uint32_t* host_row, uint32_t n_cols, const uint64_t* tab_lat,
                             const float* tab_loss, uint64_t* rng, uint64_t* event_ctr, uint8_t* status,
                             uint64_t* deliver_time, uint64_t* event_id, uint32_t* dst_order,
                             uint32_t* dst_offsets, uint64_t* min_deliver, uint64_t* min_lat, int threads) {
  uint32_t T = threads < 1 ? 1 : (threads > 64 ? 64 : (uint32_t)threads);
  ip_host* map = (ip_host*)malloc(((size_t)n_hosts + 1) * sizeof(ip_host));
  uint32_t* dst_host = (uint32_t*)malloc(((size_t)n_pkts + 1) * sizeof(uint32_t));
  uint32_t* pb = (uint32_t*)malloc((T + 1) * sizeof(uint32_t));
  uint32_t* hist = (uint32_t*)calloc((size_t)T * (n_hosts + 1), sizeof(uint32_t));
  uint64_t mind[64], minl[64];
  int64_t nd[64];
  if (!map || !dst_host || !pb || !hist) return -1;
  for (uint32_t h = 0; h < n_hosts; h++) {
    map[h].ip = host_ip[h];
    map[h].host = h;
    if (host_row[h] >= n_cols) return -1;
  }
  qsort(map, n_hosts, sizeof(ip_host), cmp_ip);
  for (uint32_t i = 0; i < n_pkts; i++)
    if (src_host[i] >= n_hosts || (i && src_host[i] < src_host[i - 1])) return -1;  /* grouped by host */
  /* T packet ranges of about equal size, cut at host boundaries */
  pb[0] = 0;
  for (uint32_t t = 1; t < T; t++) {
    uint32_t i = (uint32_t)((uint64_t)n_pkts * t / T);
    if (i < pb[t - 1]) i = pb[t - 1];
    while (i > 0 && i < n_pkts && src_host[i] == src_host[i - 1]) i++;
    pb[t] = i;
  }
  pb[T] = n_pkts;
  mt_job J = {round_end, sim_end, bootstrap_end, src_host, dst_ip, payload_len, send_time, n_hosts, n_cols,
              host_row, tab_lat, tab_loss, map, rng, event_ctr, status, deliver_time, event_id, dst_host,
              dst_offsets, dst_order, NULL, T, pb, hist, mind, minl, nd, 0};
  mt_run(&J, 0);
  if (J.err) {
    free(map);
    free(dst_host);
    free(pb);
    free(hist);
    return -2;
  }
  /* bucket offsets and each thread's start inside every bucket (thread order = packet order) */
  int64_t delivered = 0;
  uint64_t md = UINT64_MAX, ml = UINT64_MAX;
  for (uint32_t t = 0; t < T; t++) {
    delivered += nd[t];
    if (mind[t] < md) md = mind[t];
    if (minl[t] < ml) ml = minl[t];
  }
  uint32_t run = 0;
  for (uint32_t h = 0; h < n_hosts; h++) {
    dst_offsets[h] = run;
    for (uint32_t t = 0; t < T; t++) {
      const uint32_t c = hist[(size_t)t * (n_hosts + 1) + h];
      hist[(size_t)t * (n_hosts + 1) + h] = run;
      run += c;
    }
  }
  dst_offsets[n_hosts] = run;
  J.tmp = (ord_item*)malloc(((size_t)delivered + 1) * sizeof(ord_item));
  if (!J.tmp) return -1;
  mt_run(&J, 1);
  mt_run(&J, 2);
  free(J.tmp);
  free(map);
  free(dst_host);
  free(pb);
  free(hist);
  *min_deliver = md;
  *min_lat = ml;
  return delivered;
}

/* ------------------------------------------------------------------------- */
/* Multi-threaded lane baselines: the same per-host code, hosts dealt round-  */
/* robin over n_threads threads (Shadow's worker pool, thread_per_core.rs:62-64) */
/* ------------------------------------------------------------------------- */
/* off[h] = first event of host h (n_hosts + 1 entries); -4 if the events are not grouped */
static int host_offsets(const uint32_t* host, uint32_t n, uint32_t n_hosts, uint32_t* off) {
  uint32_t h = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (host[i] >= n_hosts || host[i] < (i ? host[i - 1] : 0)) return -4;
    while (h <= host[i]) off[h++] = i;
  }
  while (h <= n_hosts) off[h++] = n;
  return 0;
}

typedef struct {
  int kind; /* 0 codel, 1 inbound, 2 outbound */
  const void* a; /* the call's argument block */
  const uint32_t* off;
  uint32_t stride, phase;
  uint32_t out_begin, out_end, n_out;
  int rc;
} lane_job;

typedef struct {
  uint32_t n_hosts, cap;
  uint8_t* flags;
  uint64_t *iend, *dnext, *cur, *prev, *bytes;
  uint32_t *head, *tail, *ring_pkt;
  uint64_t* ring_ts;
  uint32_t* ring_len;
  uint32_t n_events;
  const uint32_t* host;
  const uint8_t* kind;
  const uint64_t* time;
  const uint32_t *pkt, *len;
  uint32_t* pop_result;
  uint8_t* pkt_status;
  uint32_t n_status;
} codel_call;

typedef struct {
  uint32_t n_hosts, cap;
  uint8_t* flags;
  uint64_t *iend, *dnext, *cur, *prev, *bytes;
  uint32_t *head, *tail, *ring_pkt;
  uint64_t* ring_ts;
  uint32_t* ring_len;
  uint8_t* rflags;
  uint64_t *task_time, *task_id, *task_born;
  uint32_t *cached_pkt, *cached_len;
  uint64_t *tb_cap, *tb_bal, *tb_inc, *tb_last;
  uint32_t n_arr;
  const uint32_t* host;
  const uint64_t* time;
  const uint32_t *pkt, *len;
  uint64_t window_end, bootstrap_end, sim_end;
  uint64_t *event_ctr, *fwd_time;
  uint8_t* pkt_status;
  uint32_t n_status;
} inbound_call;

static void* lane_worker(void* arg) {
  lane_job* j = (lane_job*)arg;
  if (j->kind == 0) {
    const codel_call* c = (const codel_call*)j->a;
    j->rc = codel_impl(c->n_hosts, c->cap, c->flags, c->iend, c->dnext, c->cur, c->prev, c->bytes, c->head, c->tail,
                       c->ring_pkt, c->ring_ts, c->ring_len, c->n_events, c->host, c->kind, c->time, c->pkt, c->len,
                       c->pop_result, c->pkt_status, c->n_status, j->off, j->stride, j->phase);
  } else if (j->kind == 1) {
    const inbound_call* c = (const inbound_call*)j->a;
    j->rc = inbound_impl(c->n_hosts, c->cap, c->flags, c->iend, c->dnext, c->cur, c->prev, c->bytes, c->head, c->tail,
                         c->ring_pkt, c->ring_ts, c->ring_len, c->rflags, c->task_time, c->task_id, c->task_born,
                         c->cached_pkt, c->cached_len, c->tb_cap, c->tb_bal, c->tb_inc, c->tb_last, c->n_arr, c->host,
                         c->time, c->pkt, c->len, c->window_end, c->bootstrap_end, c->sim_end, c->event_ctr,
                         c->fwd_time, c->pkt_status, c->n_status, j->off, j->stride, j->phase);
  }
  return NULL;
}

static int run_lane_jobs(lane_job* jobs, uint32_t n_threads) {
  sgo_run_threads(lane_worker, jobs, sizeof(lane_job), n_threads);
  int rc = 0;
  for (uint32_t t = 0; t < n_threads && !rc; t++) rc = jobs[t].rc;
  return rc;
}

int sgo_codel_run_mt(uint32_t n_hosts, uint32_t cap, uint8_t* flags, uint64_t* iend, uint64_t* dnext,
                     uint64_t* cur, uint64_t* prev, uint64_t* bytes, uint32_t* head, uint32_t* tail,
                     uint32_t* ring_pkt, uint64_t* ring_ts, uint32_t* ring_len, uint32_t n_events,
                     const uint32_t* host, const uint8_t* kind, const uint64_t* time, const uint32_t* pkt,
                     const uint32_t* len, uint32_t* pop_result, uint8_t* pkt_status, uint32_t n_status,
                     uint32_t n_threads) {
  if (!n_threads) return -1;
  uint32_t* off = (uint32_t*)malloc(((size_t)n_hosts + 1) * 4);
  lane_job* jobs = (lane_job*)calloc(n_threads, sizeof(lane_job));
  if (!off || !jobs) {
    free(off);
    free(jobs);
    return -1;
  }
  int rc = host_offsets(host, n_events, n_hosts, off);
  if (!rc) {
    codel_call c = {n_hosts, cap, flags, iend, dnext, cur, prev, bytes, head, tail, ring_pkt, ring_ts, ring_len,
                    n_events, host, kind, time, pkt, len, pop_result, pkt_status, n_status};
    for (uint32_t t = 0; t < n_threads; t++) jobs[t] = (lane_job){0, &c, off, n_threads, t, 0, 0, 0, 0};
    rc = run_lane_jobs(jobs, n_threads);
  }
  free(off);
  free(jobs);
  return rc;
}

int sgo_inbound_run_mt(uint32_t n_hosts, uint32_t cap, uint8_t* flags, uint64_t* iend, uint64_t* dnext,
                       uint64_t* cur, uint64_t* prev, uint64_t* bytes, uint32_t* head, uint32_t* tail,
                       uint32_t* ring_pkt, uint64_t* ring_ts, uint32_t* ring_len, uint8_t* rflags,
                       uint64_t* task_time, uint64_t* task_id, uint64_t* task_born, uint32_t* cached_pkt,
                       uint32_t* cached_len, uint64_t* tb_cap, uint64_t* tb_bal, uint64_t* tb_inc, uint64_t* tb_last,
                       uint32_t n_arr, const uint32_t* host, const uint64_t* time, const uint32_t* pkt,
                       const uint32_t* len, uint64_t window_end, uint64_t bootstrap_end, uint64_t sim_end,
                       uint64_t* event_ctr, uint64_t* fwd_time, uint8_t* pkt_status, uint32_t n_status,
                       uint32_t n_threads) {
  if (!n_threads) return -1;
  uint32_t* off = (uint32_t*)malloc(((size_t)n_hosts + 1) * 4);
  lane_job* jobs = (lane_job*)calloc(n_threads, sizeof(lane_job));
  if (!off || !jobs) {
    free(off);
    free(jobs);
    return -1;
  }
  int rc = host_offsets(host, n_arr, n_hosts, off);
  if (!rc) {
    inbound_call c = {n_hosts, cap, flags, iend, dnext, cur, prev, bytes, head, tail, ring_pkt, ring_ts, ring_len,
                      rflags, task_time, task_id, task_born, cached_pkt, cached_len, tb_cap, tb_bal, tb_inc, tb_last,
                      n_arr, host, time, pkt, len, window_end, bootstrap_end, sim_end, event_ctr, fwd_time,
                      pkt_status, n_status};
    for (uint32_t t = 0; t < n_threads; t++) jobs[t] = (lane_job){1, &c, off, n_threads, t, 0, 0, 0, 0};
    rc = run_lane_jobs(jobs, n_threads);
  }
  free(off);
  free(jobs);
  return rc;
}

/* Outbound: thread t writes its sent packets to out_* [begin_t, end_t), sized by its hosts'
 * sends plus their queued packets; *n_out = the total, out_* grouped by thread (hosts ascending
 * within a thread), each group's first slot in out_group (n_threads + 1, may be NULL). */
typedef struct {
  uint32_t n_hosts, cap;
  const uint32_t* host_ip;
  uint32_t *head, *tail, *ring_pkt, *ring_len, *ring_dst, *ring_pay;
  uint8_t* rflags;
  uint64_t *task_time, *task_id, *task_born, *tb_cap, *tb_bal, *tb_inc, *tb_last;
  uint32_t n_sends;
  const uint32_t* host;
  const uint64_t* time;
  const uint32_t *pkt, *len, *pay, *dst;
  const uint64_t *ev_id, *ev_born;
  uint64_t window_end, bootstrap_end, sim_end;
  uint64_t *event_ctr, *fwd_time;
  uint8_t* pkt_status;
  uint32_t n_status;
  uint32_t *out_host, *out_dst, *out_pay;
  uint64_t* out_time;
  uint32_t* out_pkt;
} outbound_call;

static void* outbound_worker(void* arg) {
  lane_job* j = (lane_job*)arg;
  const outbound_call* c = (const outbound_call*)j->a;
  j->rc = outbound_impl(c->n_hosts, c->cap, c->host_ip, c->head, c->tail, c->ring_pkt, c->ring_len, c->ring_dst,
                        c->ring_pay, c->rflags, c->task_time, c->task_id, c->task_born, c->tb_cap, c->tb_bal,
                        c->tb_inc, c->tb_last, c->n_sends, c->host, c->time, c->pkt, c->len, c->pay, c->dst, c->ev_id,
                        c->ev_born, c->window_end, c->bootstrap_end, c->sim_end, c->event_ctr, c->fwd_time,
                        c->pkt_status, c->n_status, c->out_host, c->out_dst, c->out_pay, c->out_time, c->out_pkt,
                        j->out_begin, j->out_end, &j->n_out, j->off, j->stride, j->phase);
  return NULL;
}

int sgo_outbound_run_mt(uint32_t n_hosts, uint32_t cap, const uint32_t* host_ip, uint32_t* head, uint32_t* tail,
                        uint32_t* ring_pkt, uint32_t* ring_len, uint32_t* ring_dst, uint32_t* ring_pay,
                        uint8_t* rflags, uint64_t* task_time, uint64_t* task_id, uint64_t* task_born, uint64_t* tb_cap,
                        uint64_t* tb_bal, uint64_t* tb_inc, uint64_t* tb_last, uint32_t n_sends, const uint32_t* host,
                        const uint64_t* time, const uint32_t* pkt, const uint32_t* len, const uint32_t* pay,
                        const uint32_t* dst, const uint64_t* ev_id, const uint64_t* ev_born, uint64_t window_end,
                        uint64_t bootstrap_end, uint64_t sim_end, uint64_t* event_ctr, uint64_t* fwd_time,
                        uint8_t* pkt_status, uint32_t n_status, uint32_t* out_host, uint32_t* out_dst,
                        uint32_t* out_pay, uint64_t* out_time, uint32_t* out_pkt, uint32_t out_cap, uint32_t* n_out,
                        uint32_t* out_group, uint32_t n_threads) {
  if (!n_threads) return -1;
  uint32_t* off = (uint32_t*)malloc(((size_t)n_hosts + 1) * 4);
  lane_job* jobs = (lane_job*)calloc(n_threads, sizeof(lane_job));
  if (!off || !jobs) {
    free(off);
    free(jobs);
    return -1;
  }
  *n_out = 0;
  int rc = host_offsets(host, n_sends, n_hosts, off);
  if (!rc) {
    outbound_call c = {n_hosts, cap, host_ip, head, tail, ring_pkt, ring_len, ring_dst, ring_pay, rflags, task_time,
                       task_id, task_born, tb_cap, tb_bal, tb_inc, tb_last, n_sends, host, time, pkt, len, pay, dst,
                       ev_id, ev_born, window_end, bootstrap_end, sim_end, event_ctr, fwd_time, pkt_status, n_status,
                       out_host, out_dst, out_pay, out_time, out_pkt};
    uint64_t at = 0;
    for (uint32_t t = 0; t < n_threads; t++) {
      uint64_t need = 0;  /* a host sends at most its queued packets and this call's sends */
      for (uint32_t h = t; h < n_hosts; h += n_threads) need += (uint64_t)(off[h + 1] - off[h]) + (tail[h] - head[h]) + 1;
      jobs[t] = (lane_job){2, &c, off, n_threads, t, (uint32_t)at, (uint32_t)(at + need < out_cap ? at + need : out_cap), 0, 0};
      at += need;
    }
    sgo_run_threads(outbound_worker, jobs, sizeof(lane_job), n_threads);
    for (uint32_t t = 0; t < n_threads && !rc; t++) rc = jobs[t].rc;
    /* compact the groups to the front */
    uint32_t w = 0;
    for (uint32_t t = 0; t < n_threads; t++) {
      if (out_group) out_group[t] = w;
      const uint32_t b = jobs[t].out_begin, k = jobs[t].n_out;
      if (b != w && k) {
        memmove(out_host + w, out_host + b, (size_t)k * 4);
        memmove(out_dst + w, out_dst + b, (size_t)k * 4);
        memmove(out_pay + w, out_pay + b, (size_t)k * 4);
        memmove(out_time + w, out_time + b, (size_t)k * 8);
        memmove(out_pkt + w, out_pkt + b, (size_t)k * 4);
      }
      w += k;
    }
    if (out_group) out_group[n_threads] = w;
    *n_out = w;
  }
  free(off);
  free(jobs);
  return rc;
}
