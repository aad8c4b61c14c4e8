/*
 * sg_faithful.c -- the reference's CPU routing build, restated cost for cost.
 *
 * TEST / BENCHMARK INFRASTRUCTURE ONLY (see sg_oracle.c's header): bench.py's
 * `cpu_baseline` leg times it beside the dense restatement (sgo_shortest_paths),
 * and tests/ check that its table equals the dense one.  The product path never
 * links or calls it.
 *
 * What it restates, step by step (Shadow 3.2.0):
 *  1. NetworkGraph::compute_shortest_paths (graph/mod.rs:183-228): for every used
 *     source, on a pool of threads (rayon's into_par_iter, :190-192),
 *     petgraph::algo::dijkstra (petgraph 0.8.1, :193-200) with its
 *     HashMap<NodeIndex, PathProperties> of scores (std SipHash-1-3), a binary
 *     heap and a visited bit set;
 *  2. .into_iter().filter(|(dst, _)| nodes.contains(dst)) -- a linear scan of the
 *     used-node slice per reached node (:203) -- collected into a per-source
 *     HashMap<(NodeIndex, NodeIndex), PathProperties> (:205-206);
 *  3. the flat_map ... collect() into one global HashMap (:190, :207-208): rayon
 *     collects the per-source maps and inserts them into one table, reserved to
 *     the total, on one thread;
 *  4. the self-pair override with the single self-loop edge (:210-217);
 *  5. generate_routing_info's remap to GML ids (sim_config.rs:423-445): the map
 *     is drained into a second HashMap<(u32, u32), PathProperties>.
 * Hash maps here are open-addressed tables with one control byte per slot (the
 * 7 top hash bits, as hashbrown keeps them) and SipHash-1-3 over the key's bytes
 * (u32 writes; std's RandomState keys are random per map, fixed here).
 * Results are identical to sgo_shortest_paths (tests/test_oracle.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
  uint64_t lat;
  float loss;
} fpp;

static inline fpp fpp_add(fpp a, uint64_t e_lat, float e_loss) { /* graph/mod.rs:322-331 */
  fpp r;
  r.lat = a.lat + e_lat;
  float oma = 1.0f - a.loss;
  float ome = 1.0f - e_loss;
  float prod = oma * ome;
  r.loss = 1.0f - prod;
  return r;
}
static inline int fpp_lt(fpp a, fpp b) { return a.lat < b.lat || (a.lat == b.lat && a.loss < b.loss); }

/* ---- SipHash-1-3 (std DefaultHasher) over 4 or 8 key bytes ---------------- */
static inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }
#define SR                                                                                           \
  do {                                                                                               \
    v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);                                        \
    v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;                                                           \
    v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;                                                           \
    v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);                                        \
  } while (0)
static const uint64_t K0 = 0x0706050403020100ull, K1 = 0x0f0e0d0c0b0a0908ull;
static inline uint64_t sip13(uint64_t m, int len) { /* len 4 or 8: one (partial) word */
  uint64_t v0 = K0 ^ 0x736f6d6570736575ull, v1 = K1 ^ 0x646f72616e646f6dull;
  uint64_t v2 = K0 ^ 0x6c7967656e657261ull, v3 = K1 ^ 0x7465646279746573ull;
  uint64_t b = ((uint64_t)len << 56);
  if (len == 8) {
    v3 ^= m;
    SR;
    v0 ^= m;
  } else {
    b |= m;
  }
  v3 ^= b;
  SR;
  v0 ^= b;
  v2 ^= 0xff;
  SR;
  SR;
  SR;
  return v0 ^ v1 ^ v2 ^ v3;
}

/* ---- open-addressed map u64 key -> fpp, control bytes ----------------------- */
typedef struct {
  uint64_t key;
  fpp val;
} fslot;
typedef struct {
  uint8_t* ctrl; /* 0x80 empty, else the hash's top 7 bits */
  fslot* s;
  size_t cap, len; /* cap a power of two; grows at 7/8 */
  int key_len;     /* 4 (node) or 8 (pair) */
} fmap;

static int fmap_init(fmap* m, size_t want, int key_len) {
  size_t cap = 8;
  while (cap * 7 / 8 < want) cap <<= 1;
  m->ctrl = (uint8_t*)malloc(cap);
  m->s = (fslot*)malloc(cap * sizeof(fslot));
  if (!m->ctrl || !m->s) return -1;
  memset(m->ctrl, 0x80, cap);
  m->cap = cap;
  m->len = 0;
  m->key_len = key_len;
  return 0;
}
static void fmap_free(fmap* m) {
  free(m->ctrl);
  free(m->s);
  m->ctrl = NULL;
  m->s = NULL;
}
/* slot of key (existing or the empty one to fill) */
static inline size_t fmap_find(const fmap* m, uint64_t key, uint64_t h) {
  const uint8_t h2 = (uint8_t)(h >> 57);
  size_t i = (size_t)h & (m->cap - 1);
  for (;;) {
    const uint8_t c = m->ctrl[i];
    if (c == 0x80) return i;
    if (c == h2 && m->s[i].key == key) return i;
    i = (i + 1) & (m->cap - 1);
  }
}
static int fmap_grow(fmap* m) {
  fmap n;
  if (fmap_init(&n, m->cap, m->key_len)) return -1; /* doubles */
  for (size_t i = 0; i < m->cap; i++)
    if (m->ctrl[i] != 0x80) {
      const uint64_t h = sip13(m->s[i].key, m->key_len);
      const size_t j = fmap_find(&n, m->s[i].key, h);
      n.ctrl[j] = (uint8_t)(h >> 57);
      n.s[j] = m->s[i];
      n.len++;
    }
  fmap_free(m);
  *m = n;
  return 0;
}
/* returns the slot; *fresh = 1 if it was vacant (now occupied, value unset) */
static inline fslot* fmap_entry(fmap* m, uint64_t key, int* fresh) {
  if ((m->len + 1) > m->cap * 7 / 8 && fmap_grow(m)) return NULL;
  const uint64_t h = sip13(key, m->key_len);
  const size_t i = fmap_find(m, key, h);
  *fresh = m->ctrl[i] == 0x80;
  if (*fresh) {
    m->ctrl[i] = (uint8_t)(h >> 57);
    m->s[i].key = key;
    m->len++;
  }
  return &m->s[i];
}
static inline const fslot* fmap_get(const fmap* m, uint64_t key) {
  const size_t i = fmap_find(m, key, sip13(key, m->key_len));
  return m->ctrl[i] == 0x80 ? NULL : &m->s[i];
}

/* ---- petgraph adjacency (as sg_oracle.c adj_build) --------------------------- */
typedef struct {
  uint32_t *off, *dst, *edge;
} fadj;

/* ---- binary heap of MinScored(score, node) ---------------------------------- */
typedef struct {
  fpp k;
  uint32_t node;
} fhi;
typedef struct {
  fhi* a;
  size_t n, cap;
} fheap;
static int fheap_push(fheap* h, fpp k, uint32_t node) {
  if (h->n == h->cap) {
    size_t nc = h->cap ? 2 * h->cap : 64;
    fhi* na = (fhi*)realloc(h->a, nc * sizeof(fhi));
    if (!na) return -1;
    h->a = na;
    h->cap = nc;
  }
  size_t i = h->n++;
  fhi x = {k, node};
  while (i) {
    size_t p = (i - 1) / 2;
    if (!fpp_lt(x.k, h->a[p].k)) break;
    h->a[i] = h->a[p];
    i = p;
  }
  h->a[i] = x;
  return 0;
}
static fhi fheap_pop(fheap* h) {
  fhi top = h->a[0], x = h->a[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    fpp mk = x.k;
    if (l < h->n && fpp_lt(h->a[l].k, mk)) m = l, mk = h->a[l].k;
    if (r < h->n && fpp_lt(h->a[r].k, mk)) m = r;
    if (m == i) break;
    h->a[i] = h->a[m];
    i = m;
  }
  if (h->n) h->a[i] = x;
  return top;
}

typedef struct {
  const fadj* A;
  const uint64_t* elat;
  const float* eloss;
  const uint32_t* used;
  uint32_t n, n_used, rows;
  fmap* per_src; /* rows maps, (src, dst) -> path */
  uint32_t next;
  pthread_mutex_t mu;
  int err;
} fjob;

static void* fworker(void* p) {
  fjob* J = (fjob*)p;
  uint8_t* visited = (uint8_t*)malloc(J->n);
  fheap hp = {0, 0, 0};
  for (;;) {
    pthread_mutex_lock(&J->mu);
    const uint32_t r = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (r >= J->rows || !visited) break;
    const uint32_t s = J->used[r];
    /* petgraph::algo::dijkstra: scores HashMap, BinaryHeap, visited set */
    memset(visited, 0, J->n);
    fmap scores;
    if (fmap_init(&scores, 0, 4)) {
      J->err = 1;
      break;
    }
    int fresh;
    fslot* e = fmap_entry(&scores, s, &fresh);
    e->val = (fpp){0, 0.0f};
    hp.n = 0;
    fheap_push(&hp, e->val, s);
    while (hp.n) {
      const fhi it = fheap_pop(&hp);
      if (visited[it.node]) continue;
      for (uint32_t k = J->A->off[it.node]; k < J->A->off[it.node + 1]; k++) {
        const uint32_t nx = J->A->dst[k];
        if (visited[nx]) continue;
        const uint32_t ed = J->A->edge[k];
        const fpp ns = fpp_add(it.k, J->elat[ed], J->eloss[ed]);
        fslot* sl = fmap_entry(&scores, nx, &fresh);
        if (!sl) {
          J->err = 1;
          break;
        }
        if (fresh || fpp_lt(ns, sl->val)) {
          sl->val = ns;
          fheap_push(&hp, ns, nx);
        }
      }
      visited[it.node] = 1;
    }
    /* .into_iter().filter(|(dst, _)| nodes.contains(dst)).map(..).collect::<HashMap<_, _>>() */
    fmap* out = &J->per_src[r];
    if (fmap_init(out, 0, 8)) {
      J->err = 1;
      fmap_free(&scores);
      break;
    }
    for (size_t i = 0; i < scores.cap; i++) {
      if (scores.ctrl[i] == 0x80) continue;
      const uint32_t d = (uint32_t)scores.s[i].key;
      int in = 0;
      for (uint32_t j = 0; j < J->n_used; j++) /* slice::contains */
        if (J->used[j] == d) {
          in = 1;
          break;
        }
      if (!in) continue;
      fslot* o = fmap_entry(out, ((uint64_t)d << 32) | s, &fresh);
      o->val = scores.s[i].val;
    }
    fmap_free(&scores);
  }
  free(visited);
  free(hp.a);
  return NULL;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

/*
 * Rows [0, rows) of compute_shortest_paths + generate_routing_info as the
 * reference builds them.  node_id[v] = the GML id of node index v.  Timings (s)
 * into t_phase: [0] per-source Dijkstra + filter + per-source maps (threads),
 * [1] the global collect, [2] the self-pair override, [3] the id remap.
 * out_lat / out_loss (rows x n_used, may be NULL): read back from the final map
 * (untimed) for the parity check.  Returns 0, or 1 on allocation failure, 2 on a
 * missing self-loop.
 */
int sgo_routing_faithful(uint32_t n, uint32_t m, const uint32_t* esrc, const uint32_t* edst, const uint64_t* elat,
                         const float* eloss, int directed, const uint32_t* used, uint32_t n_used, uint32_t rows,
                         const uint32_t* node_id, int n_threads, double* t_phase, uint64_t* out_lat,
                         float* out_loss) {
  if (rows > n_used) return 1;
  fadj A;
  A.off = (uint32_t*)calloc((size_t)n + 1, 4);
  const size_t cap = directed ? m : 2 * (size_t)m;
  A.dst = (uint32_t*)malloc((cap + 1) * 4);
  A.edge = (uint32_t*)malloc((cap + 1) * 4);
  uint32_t* cur = (uint32_t*)malloc(((size_t)n + 1) * 4);
  if (!A.off || !A.dst || !A.edge || !cur) return 1;
  for (uint32_t i = 0; i < m; i++) {
    A.off[esrc[i] + 1]++;
    if (!directed && esrc[i] != edst[i]) A.off[edst[i] + 1]++;
  }
  for (uint32_t v = 0; v < n; v++) A.off[v + 1] += A.off[v];
  memcpy(cur, A.off, ((size_t)n + 1) * 4);
  for (uint32_t i = 0; i < m; i++) {
    const uint32_t s = esrc[i], d = edst[i];
    A.dst[cur[s]] = d;
    A.edge[cur[s]++] = i;
    if (!directed && s != d) {
      A.dst[cur[d]] = s;
      A.edge[cur[d]++] = i;
    }
  }
  free(cur);
  fjob J;
  memset(&J, 0, sizeof(J));
  J.A = &A;
  J.elat = elat;
  J.eloss = eloss;
  J.used = used;
  J.n = n;
  J.n_used = n_used;
  J.rows = rows;
  J.per_src = (fmap*)calloc(rows ? rows : 1, sizeof(fmap));
  pthread_mutex_init(&J.mu, NULL);
  int T = n_threads < 1 ? 1 : n_threads;
  double t0 = now_s();
  pthread_t* th = (pthread_t*)malloc((size_t)T * sizeof(pthread_t));
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, fworker, &J);
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  free(th);
  double t1 = now_s();
  int rc = J.err ? 1 : 0;
  /* global collect: reserve the total, insert every per-source entry on one thread */
  size_t total = 0;
  for (uint32_t r = 0; r < rows; r++) total += J.per_src[r].len;
  fmap g;
  if (!rc && fmap_init(&g, total, 8)) rc = 1;
  for (uint32_t r = 0; !rc && r < rows; r++) {
    fmap* p = &J.per_src[r];
    for (size_t i = 0; i < p->cap; i++)
      if (p->ctrl[i] != 0x80) {
        int fresh;
        fslot* o = fmap_entry(&g, p->s[i].key, &fresh);
        if (!o) {
          rc = 1;
          break;
        }
        o->val = p->s[i].val;
      }
    fmap_free(p);
  }
  double t2 = now_s();
  /* self pairs := the single self-loop edge (graph/mod.rs:210-217) */
  for (uint32_t j = 0; !rc && j < rows; j++) {
    const uint32_t u = used[j];
    uint32_t c = 0, e = 0;
    for (uint32_t k = A.off[u]; k < A.off[u + 1]; k++)
      if (A.dst[k] == u) {
        if (!c) e = A.edge[k];
        c++;
      }
    if (c != 1) {
      rc = 2;
      break;
    }
    int fresh;
    fslot* o = fmap_entry(&g, ((uint64_t)u << 32) | u, &fresh);
    o->val = (fpp){elat[e], eloss[e]};
  }
  double t3 = now_s();
  /* generate_routing_info: into_iter().map(to_ids).collect() into a second map */
  fmap ids;
  if (!rc && fmap_init(&ids, g.len, 8)) rc = 1;
  for (size_t i = 0; !rc && i < g.cap; i++)
    if (g.ctrl[i] != 0x80) {
      const uint32_t s = (uint32_t)g.s[i].key, d = (uint32_t)(g.s[i].key >> 32);
      int fresh;
      fslot* o = fmap_entry(&ids, ((uint64_t)node_id[d] << 32) | node_id[s], &fresh);
      o->val = g.s[i].val;
    }
  double t4 = now_s();
  if (!rc) fmap_free(&g);
  if (t_phase) {
    t_phase[0] = t1 - t0;
    t_phase[1] = t2 - t1;
    t_phase[2] = t3 - t2;
    t_phase[3] = t4 - t3;
  }
  if (!rc && out_lat && out_loss) /* RoutingInfo::path per (row, col), untimed */
    for (uint32_t i = 0; i < rows; i++)
      for (uint32_t j = 0; j < n_used; j++) {
        const fslot* o = fmap_get(&ids, ((uint64_t)node_id[used[j]] << 32) | node_id[used[i]]);
        out_lat[(size_t)i * n_used + j] = o ? o->val.lat : UINT64_MAX;
        out_loss[(size_t)i * n_used + j] = o ? o->val.loss : -1.0f;
      }
  if (!rc) fmap_free(&ids);
  free(J.per_src);
  pthread_mutex_destroy(&J.mu);
  free(A.off);
  free(A.dst);
  free(A.edge);
  return rc;
}
