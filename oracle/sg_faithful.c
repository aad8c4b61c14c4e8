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
 *
 * sgo_deliver_faithful (below) does the same for the delivery round.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void sgo_run_threads(void* (*fn)(void*), void* args, size_t stride, uint32_t n); /* sg_oracle.c */

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
  sgo_run_threads(fworker, &J, 0, (uint32_t)T);
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

/* ========================================================================== */
/* The reference's delivery round, cost for cost                               */
/* ========================================================================== */
/*
 * Worker::send_packet (worker.rs:322-397) on the reference's data structures:
 *  - Dns::addr_to_host_id (dns.rs:176-178): HashMap<Ipv4Addr, Record> lookup;
 *  - WorkerShared::reliability and ::latency (worker.rs:517-535): each does two
 *    IpAssignment::get_node lookups (HashMap<IpAddr, u32>, graph/mod.rs:391-393)
 *    and a RoutingInfo::path lookup (HashMap<(u32, u32), PathProperties> holding
 *    every node pair, graph/mod.rs:445-447);
 *  - increment_packet_count (worker.rs:541-546, graph/mod.rs:449-456): two more
 *    get_node lookups, then a write lock on one global RwLock<HashMap<(u32, u32),
 *    u64>> and an entry update;
 *  - push_packet_to_host (worker.rs:597-607): HashMap<HostId, Arc<Mutex<
 *    EventQueue>>> lookup, the queue's mutex, a BinaryHeap push (event_queue.rs:
 *    31-37) ordered as Event (event.rs:84-155: time, then source host, then the
 *    source's event id).
 * Worker threads take hosts round-robin (thread_per_core.rs:62-64); a host's
 * packets run in order on its thread.  The maps are built before the round
 * (untimed: the reference builds them at startup); the round is timed.  The
 * per-destination heaps are popped afterwards (untimed) into dst_order /
 * dst_offsets, so tests compare the whole round with sgo_deliver_round.
 * Keys are hashed as 4 or 8 bytes (std also hashes an IpAddr's discriminant).
 */
double sgo_xoshiro_next_f64(uint64_t s[4]);
/* statuses as sg_oracle.c SGO_ST_* (PacketStatus outcomes of send_packet) */
enum { SGO_ST_DELIVERED_F = 0, SGO_ST_DROP_LOSS_F = 1, SGO_ST_NO_DST_F = 2, SGO_ST_SIM_END_F = 3 };

typedef struct {
  uint64_t time, eid;
  uint32_t src, pkt;
} fev;
static inline int fev_lt(const fev* a, const fev* b) {
  if (a->time != b->time) return a->time < b->time;
  if (a->src != b->src) return a->src < b->src;
  return a->eid < b->eid;
}
typedef struct {
  pthread_mutex_t mu;
  fev* a;
  uint32_t n, cap;
} fqueue;
static int fqueue_push(fqueue* q, fev e) { /* min-heap (BinaryHeap<Reverse<Event>>) */
  if (q->n == q->cap) {
    const uint32_t nc = q->cap ? 2 * q->cap : 8;
    fev* na = (fev*)realloc(q->a, (size_t)nc * sizeof(fev));
    if (!na) return -1;
    q->a = na;
    q->cap = nc;
  }
  uint32_t i = q->n++;
  while (i) {
    const uint32_t p = (i - 1) / 2;
    if (!fev_lt(&e, &q->a[p])) break;
    q->a[i] = q->a[p];
    i = p;
  }
  q->a[i] = e;
  return 0;
}
static fev fqueue_pop(fqueue* q) {
  const fev top = q->a[0], last = q->a[--q->n];
  uint32_t i = 0;
  for (;;) {
    uint32_t c = 2 * i + 1;
    if (c >= q->n) break;
    if (c + 1 < q->n && fev_lt(&q->a[c + 1], &q->a[c])) c++;
    if (!fev_lt(&q->a[c], &last)) break;
    q->a[i] = q->a[c];
    i = c;
  }
  if (q->n) q->a[i] = last;
  return top;
}

typedef struct {
  /* inputs */
  uint64_t round_end, sim_end, bootstrap_end;
  const uint32_t *src_host, *dst_ip, *payload_len;
  const uint64_t* send_time;
  const uint32_t* host_ip;
  uint32_t n_hosts;
  const uint32_t* host_first; /* per host: first packet (n_hosts + 1) */
  uint64_t *rng, *event_ctr;
  /* the reference's structures */
  fmap dns, ipa, paths, queues_idx, counters;
  pthread_rwlock_t counters_lock;
  fqueue* queues;
  /* outputs */
  uint8_t* status;
  uint64_t *deliver_time, *event_id;
  uint32_t T;
  uint64_t mind[64], minl[64];
  int64_t delivered[64];
  int err;
} fdjob;
typedef struct {
  fdjob* J;
  uint32_t t;
} fdarg;

static void* fdworker(void* p) {
  fdarg* A = (fdarg*)p;
  fdjob* J = A->J;
  uint64_t mind = UINT64_MAX, minl = UINT64_MAX;
  int64_t nd = 0;
  for (uint32_t h = A->t; h < J->n_hosts; h += J->T) /* round-robin hosts */
    for (uint32_t i = J->host_first[h]; i < J->host_first[h + 1]; i++) {
      const uint64_t now = J->send_time[i];
      J->deliver_time[i] = 0;
      J->event_id[i] = UINT64_MAX;
      if (now >= J->sim_end) {
        J->status[i] = SGO_ST_SIM_END_F;
        continue;
      }
      const uint32_t src_ip = J->host_ip[h], dst_ip = J->dst_ip[i];
      const fslot* dh = fmap_get(&J->dns, dst_ip); /* resolve_ip_to_host_id */
      if (!dh) {
        J->status[i] = SGO_ST_NO_DST_F;
        continue;
      }
      const uint32_t d = (uint32_t)dh->val.lat;
      /* reliability(): two get_node + path */
      uint64_t sn = fmap_get(&J->ipa, src_ip)->val.lat, dn = fmap_get(&J->ipa, dst_ip)->val.lat;
      const fslot* pp = fmap_get(&J->paths, (dn << 32) | sn);
      const double reliability = (double)(1.0f - pp->val.loss);
      const double chance = sgo_xoshiro_next_f64(&J->rng[4 * (size_t)h]);
      if (!(now < J->bootstrap_end) && chance >= reliability && J->payload_len[i] > 0) {
        J->status[i] = SGO_ST_DROP_LOSS_F;
        continue;
      }
      /* latency(): two get_node + path, again */
      sn = fmap_get(&J->ipa, src_ip)->val.lat;
      dn = fmap_get(&J->ipa, dst_ip)->val.lat;
      const uint64_t delay = fmap_get(&J->paths, (dn << 32) | sn)->val.lat;
      if (delay < minl) minl = delay;
      /* increment_packet_count(): two get_node + the global write lock */
      sn = fmap_get(&J->ipa, src_ip)->val.lat;
      dn = fmap_get(&J->ipa, dst_ip)->val.lat;
      pthread_rwlock_wrlock(&J->counters_lock);
      int fresh;
      fslot* c = fmap_entry(&J->counters, (dn << 32) | sn, &fresh);
      if (!c) J->err = 1;
      else c->val.lat = fresh ? 1 : (c->val.lat == UINT64_MAX ? UINT64_MAX : c->val.lat + 1);
      pthread_rwlock_unlock(&J->counters_lock);
      uint64_t tt = now + delay;
      if (tt < now || tt == UINT64_MAX) {
        J->err = 2;
        tt = UINT64_MAX - 1;
      }
      if (tt < J->round_end) tt = J->round_end;
      if (tt < mind) mind = tt;
      J->status[i] = SGO_ST_DELIVERED_F;
      J->deliver_time[i] = tt;
      const uint64_t eid = J->event_ctr[h]++;
      J->event_id[i] = eid;
      /* push_packet_to_host(): queue lookup, its mutex, the heap push */
      fqueue* q = &J->queues[fmap_get(&J->queues_idx, d)->val.lat];
      pthread_mutex_lock(&q->mu);
      if (fqueue_push(q, (fev){tt, eid, h, i})) J->err = 1;
      pthread_mutex_unlock(&q->mu);
      nd++;
    }
  J->mind[A->t] = mind;
  J->minl[A->t] = minl;
  J->delivered[A->t] = nd;
  return NULL;
}

/*
 * One round over packets grouped by source host.  host_node[h] = the routing
 * node (table row and column) of host h; the table is n_nodes x n_nodes.
 * t_setup / t_round: seconds spent building the maps and in the round.  Returns
 * the delivered count, -1 on bad input or allocation failure, -2 on arrival-time
 * overflow.
 */
int64_t sgo_deliver_faithful(uint64_t round_end, uint64_t sim_end, uint64_t bootstrap_end, uint32_t n_pkts,
                             const uint32_t* src_host, const uint32_t* dst_ip, const uint32_t* payload_len,
                             const uint64_t* send_time, uint32_t n_hosts, const uint32_t* host_ip,
                             const uint32_t* host_node, uint32_t n_nodes, const uint64_t* tab_lat,
                             const float* tab_loss, uint64_t* rng, uint64_t* event_ctr, uint8_t* status,
                             uint64_t* deliver_time, uint64_t* event_id, uint32_t* dst_order, uint32_t* dst_offsets,
                             uint64_t* min_deliver, uint64_t* min_lat, int threads, double* t_setup,
                             double* t_round) {
  fdjob* J = (fdjob*)calloc(1, sizeof(fdjob));
  if (!J) return -1;
  const double t0 = now_s();
  J->T = threads < 1 ? 1 : (threads > 64 ? 64 : (uint32_t)threads);
  J->round_end = round_end;
  J->sim_end = sim_end;
  J->bootstrap_end = bootstrap_end;
  J->src_host = src_host;
  J->dst_ip = dst_ip;
  J->payload_len = payload_len;
  J->send_time = send_time;
  J->host_ip = host_ip;
  J->n_hosts = n_hosts;
  J->rng = rng;
  J->event_ctr = event_ctr;
  J->status = status;
  J->deliver_time = deliver_time;
  J->event_id = event_id;
  int64_t rc = 0;
  uint32_t* first = (uint32_t*)calloc((size_t)n_hosts + 1, 4);
  J->queues = (fqueue*)calloc(n_hosts ? n_hosts : 1, sizeof(fqueue));
  if (!first || !J->queues) rc = -1;
  for (uint32_t i = 0; !rc && i < n_pkts; i++) {
    if (src_host[i] >= n_hosts || (i && src_host[i] < src_host[i - 1])) rc = -1;
    else first[src_host[i] + 1]++;
  }
  for (uint32_t h = 0; !rc && h < n_hosts; h++) {
    first[h + 1] += first[h];
    if (host_node[h] >= n_nodes) rc = -1;
  }
  J->host_first = first;
  /* Dns and IpAssignment: one entry per host */
  if (!rc && (fmap_init(&J->dns, n_hosts, 4) || fmap_init(&J->ipa, n_hosts, 4) ||
              fmap_init(&J->queues_idx, n_hosts, 4) || fmap_init(&J->counters, 1024, 8)))
    rc = -1;
  for (uint32_t h = 0; !rc && h < n_hosts; h++) {
    int fresh;
    fslot* s = fmap_entry(&J->dns, host_ip[h], &fresh);
    if (!s || !fresh) {
      rc = -1;
      break;
    }
    s->val.lat = h;
    s = fmap_entry(&J->ipa, host_ip[h], &fresh);
    s->val.lat = host_node[h];
    s = fmap_entry(&J->queues_idx, h, &fresh);
    s->val.lat = h;
    pthread_mutex_init(&J->queues[h].mu, NULL);
  }
  /* RoutingInfo paths: every node pair */
  if (!rc && fmap_init(&J->paths, (size_t)n_nodes * n_nodes, 8)) rc = -1;
  for (uint32_t a = 0; !rc && a < n_nodes; a++)
    for (uint32_t b = 0; b < n_nodes; b++) {
      int fresh;
      fslot* s = fmap_entry(&J->paths, ((uint64_t)b << 32) | a, &fresh);
      if (!s) {
        rc = -1;
        break;
      }
      s->val = (fpp){tab_lat[(size_t)a * n_nodes + b], tab_loss[(size_t)a * n_nodes + b]};
    }
  pthread_rwlock_init(&J->counters_lock, NULL);
  const double t1 = now_s();
  double t2 = t1;
  if (!rc) {
    fdarg args[64];
    for (uint32_t t = 0; t < J->T; t++) args[t] = (fdarg){J, t};
    sgo_run_threads(fdworker, args, sizeof(fdarg), J->T);
    t2 = now_s();
    if (J->err) rc = J->err == 2 ? -2 : -1;
  }
  if (!rc) { /* the destinations' queues, popped in order (untimed) */
    int64_t nd = 0;
    uint64_t md = UINT64_MAX, ml = UINT64_MAX;
    for (uint32_t t = 0; t < J->T; t++) {
      nd += J->delivered[t];
      if (J->mind[t] < md) md = J->mind[t];
      if (J->minl[t] < ml) ml = J->minl[t];
    }
    uint32_t k = 0;
    for (uint32_t h = 0; h < n_hosts; h++) {
      dst_offsets[h] = k;
      while (J->queues[h].n) dst_order[k++] = fqueue_pop(&J->queues[h]).pkt;
    }
    dst_offsets[n_hosts] = k;
    *min_deliver = md;
    *min_lat = ml;
    rc = nd;
  }
  if (t_setup) *t_setup = t1 - t0;
  if (t_round) *t_round = t2 - t1;
  for (uint32_t h = 0; J->queues && h < n_hosts; h++) {
    free(J->queues[h].a);
    pthread_mutex_destroy(&J->queues[h].mu);
  }
  free(J->queues);
  if (J->dns.ctrl) fmap_free(&J->dns);
  if (J->ipa.ctrl) fmap_free(&J->ipa);
  if (J->queues_idx.ctrl) fmap_free(&J->queues_idx);
  if (J->counters.ctrl) fmap_free(&J->counters);
  if (J->paths.ctrl) fmap_free(&J->paths);
  pthread_rwlock_destroy(&J->counters_lock);
  free(first);
  free(J);
  return rc;
}
