/*
 * tswap_oracle.c — TEST INFRASTRUCTURE ONLY (see tswap_oracle.h).
 *
 * Faithful single-threaded CPU restatement of the reference planning path,
 * RenKoya1/p2p_distributed_tswap @ 2025-11-21, src/algorithm/tswap.rs.
 * "parity unpinned": no Rust toolchain here and no reference fixtures; the
 * restatement is cross-checked by oracle/py_restatement.py.
 *
 * Every function cites the reference lines it restates. Data-structure
 * choices (dense stamped arrays instead of HashMap, cell index instead of
 * node id) do not change any result: HashMap iteration order is never
 * consulted on this path.
 */
#include "tswap_oracle.h"

#include <stdlib.h>
#include <string.h>

enum { DIR_S = 0, DIR_E = 1, DIR_N = 2, DIR_W = 3 };
/* neighbour order (dx,dy) = (0,1),(1,0),(0,-1),(-1,0): tswap.rs:62 */
static const int DX[4] = {0, 1, 0, -1};
static const int DY[4] = {1, 0, -1, 0};

typedef struct {
    uint32_t node, g, f;
} anode; /* AstarNode, tswap.rs:293-298 */

struct orc_graph {
    uint32_t w, h, ncell;
    uint8_t *free_;    /* 1 = not '@' (tswap.rs:53) */
    uint32_t *nb;      /* 4 per cell, UINT32_MAX = absent */
    uint8_t *nbn;      /* number of neighbours */
    /* A* scratch (stand-in for the per-call HashMaps g_score / came_from) */
    uint32_t *gs_stamp, *gs_val, *came;
    uint32_t stamp;
    anode *heap;
    size_t heap_len, heap_cap;
    uint64_t calls, pops;
};

orc_graph *orc_graph_create(const uint8_t *cells, uint32_t w, uint32_t h) {
    if (!cells || w == 0 || h == 0) return NULL;
    orc_graph *gr = (orc_graph *)calloc(1, sizeof(orc_graph));
    gr->w = w;
    gr->h = h;
    gr->ncell = w * h;
    gr->free_ = (uint8_t *)malloc(gr->ncell);
    gr->nb = (uint32_t *)malloc(sizeof(uint32_t) * 4 * gr->ncell);
    gr->nbn = (uint8_t *)calloc(gr->ncell, 1);
    gr->gs_stamp = (uint32_t *)calloc(gr->ncell, sizeof(uint32_t));
    gr->gs_val = (uint32_t *)malloc(sizeof(uint32_t) * gr->ncell);
    gr->came = (uint32_t *)malloc(sizeof(uint32_t) * gr->ncell);
    gr->heap_cap = 1024;
    gr->heap = (anode *)malloc(sizeof(anode) * gr->heap_cap);
    for (uint32_t c = 0; c < gr->ncell; c++) gr->free_[c] = (cells[c] != '@');
    /* tswap.rs:60-77: neighbours of each free cell, in S,E,N,W order */
    for (uint32_t y = 0; y < h; y++)
        for (uint32_t x = 0; x < w; x++) {
            uint32_t c = y * w + x;
            uint8_t k = 0;
            for (int d = 0; d < 4; d++) gr->nb[4 * c + d] = UINT32_MAX;
            if (!gr->free_[c]) continue;
            for (int d = 0; d < 4; d++) {
                long nx = (long)x + DX[d], ny = (long)y + DY[d];
                if (nx < 0 || ny < 0 || nx >= (long)w || ny >= (long)h) continue;
                uint32_t nc = (uint32_t)ny * w + (uint32_t)nx;
                if (gr->free_[nc]) gr->nb[4 * c + k++] = nc;
            }
            gr->nbn[c] = k;
        }
    return gr;
}

void orc_graph_destroy(orc_graph *gr) {
    if (!gr) return;
    free(gr->free_);
    free(gr->nb);
    free(gr->nbn);
    free(gr->gs_stamp);
    free(gr->gs_val);
    free(gr->came);
    free(gr->heap);
    free(gr);
}

uint64_t orc_stat_calls(orc_graph *gr) { return gr->calls; }
uint64_t orc_stat_pops(orc_graph *gr) { return gr->pops; }

/* ---- Rust std::collections::BinaryHeap<AstarNode>, restated ------------
 * Ord (tswap.rs:314-321): other.f.cmp(self.f).then(other.g.cmp(self.g)),
 * i.e. a > b  <=>  a.f < b.f || (a.f == b.f && a.g < b.g).  `<=` is !(>).
 * push  = Vec::push + sift_up(0, old_len)
 * pop   = Vec::pop; if non-empty: swap with data[0], sift_down_to_bottom(0)
 * sift_up: move hole up while !(elem <= parent)
 * sift_down_to_bottom: move hole to the greater child (right when
 *   left <= right) while child <= end-2; then to child if child == end-1;
 *   then sift_up(start, pos).                                              */
static inline int an_gt(anode a, anode b) {
    return a.f < b.f || (a.f == b.f && a.g < b.g);
}
static inline int an_le(anode a, anode b) { return !an_gt(a, b); }

static size_t heap_sift_up(orc_graph *gr, size_t start, size_t pos) {
    anode *d = gr->heap;
    anode elem = d[pos];
    while (pos > start) {
        size_t parent = (pos - 1) / 2;
        if (an_le(elem, d[parent])) break;
        d[pos] = d[parent];
        pos = parent;
    }
    d[pos] = elem;
    return pos;
}

static void heap_push(orc_graph *gr, anode item) {
    if (gr->heap_len == gr->heap_cap) {
        gr->heap_cap *= 2;
        gr->heap = (anode *)realloc(gr->heap, sizeof(anode) * gr->heap_cap);
    }
    size_t old_len = gr->heap_len;
    gr->heap[gr->heap_len++] = item;
    heap_sift_up(gr, 0, old_len);
}

static void heap_sift_down_to_bottom(orc_graph *gr, size_t pos) {
    anode *d = gr->heap;
    size_t end = gr->heap_len, start = pos;
    anode elem = d[pos];
    size_t child = 2 * pos + 1;
    size_t lim = end >= 2 ? end - 2 : 0; /* end.saturating_sub(2) */
    while (child <= lim) {
        child += an_le(d[child], d[child + 1]) ? 1 : 0;
        d[pos] = d[child];
        pos = child;
        child = 2 * pos + 1;
    }
    if (child == end - 1) {
        d[pos] = d[child];
        pos = child;
    }
    d[pos] = elem;
    heap_sift_up(gr, start, pos);
}

static int heap_pop(orc_graph *gr, anode *out) {
    if (gr->heap_len == 0) return 0;
    anode item = gr->heap[--gr->heap_len];
    if (gr->heap_len > 0) {
        anode t = gr->heap[0];
        gr->heap[0] = item;
        item = t;
        heap_sift_down_to_bottom(gr, 0);
    }
    *out = item;
    return 1;
}

static inline uint32_t manhattan(const orc_graph *gr, uint32_t a, uint32_t b) {
    long ax = a % gr->w, ay = a / gr->w, bx = b % gr->w, by = b / gr->w;
    long dx = ax - bx, dy = ay - by;
    return (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
}

/* get_path, tswap.rs:288-390 */
int32_t orc_get_path_next(orc_graph *gr, uint32_t start, uint32_t goal,
                          uint32_t *next, uint64_t *pops_out) {
    gr->calls++;
    if (start == goal) { /* :289-291 */
        *next = start;
        if (pops_out) *pops_out = 0;
        return 1;
    }
    if (++gr->stamp == 0) { /* stamp wrap: clear */
        memset(gr->gs_stamp, 0, sizeof(uint32_t) * gr->ncell);
        gr->stamp = 1;
    }
    const uint32_t st = gr->stamp;
    uint64_t pops = 0;
    gr->heap_len = 0;
    /* :333-339 */
    gr->gs_stamp[start] = st;
    gr->gs_val[start] = 0;
    anode s = {start, 0, manhattan(gr, start, goal)};
    heap_push(gr, s);
    anode cur;
    while (heap_pop(gr, &cur)) { /* :341 */
        pops++;
        uint32_t cid = cur.node;
        if (cid == goal) { /* :344-355 — rebuild via came_from */
            uint32_t c = cid;
            int32_t len = 1;
            while (gr->came[c] != start) {
                c = gr->came[c];
                len++;
            }
            *next = c;
            gr->pops += pops;
            if (pops_out) *pops_out = pops;
            return len + 1;
        }
        for (uint32_t k = 0; k < gr->nbn[cid]; k++) { /* :357-375 */
            uint32_t nbid = gr->nb[4 * cid + k];
            uint32_t tg = cur.g + 1;
            uint32_t old = gr->gs_stamp[nbid] == st ? gr->gs_val[nbid] : UINT32_MAX;
            if (tg < old) {
                gr->came[nbid] = cid;
                gr->gs_stamp[nbid] = st;
                gr->gs_val[nbid] = tg;
                anode e = {nbid, tg, tg + manhattan(gr, nbid, goal)};
                heap_push(gr, e);
            }
        }
    }
    /* :378-389 — unreachable: first neighbour strictly closer in Manhattan */
    uint32_t best = start, mind = manhattan(gr, start, goal);
    for (uint32_t k = 0; k < gr->nbn[start]; k++) {
        uint32_t nbid = gr->nb[4 * start + k];
        uint32_t d = manhattan(gr, nbid, goal);
        if (d < mind) {
            mind = d;
            best = nbid;
        }
    }
    *next = best;
    gr->pops += pops;
    if (pops_out) *pops_out = pops;
    return 2;
}

/* Next-hop code of get_path(c, goal) for every free cell c (0..3 = S,E,N,W neighbour,
 * 4 = path[1] == c, i.e. c == goal or the fallback found no closer neighbour);
 * blocked cells get 0xFF. Checker for the device next-hop tables. */
int orc_next_codes(orc_graph *gr, uint32_t goal, uint8_t *out) {
    if (goal >= gr->ncell || !gr->free_[goal]) return -1;
    for (uint32_t c = 0; c < gr->ncell; c++) {
        if (!gr->free_[c]) {
            out[c] = 0xFF;
            continue;
        }
        uint32_t nx;
        orc_get_path_next(gr, c, goal, &nx, NULL);
        if (nx == c) out[c] = 4;
        else if (nx == c + gr->w) out[c] = 0;
        else if (nx == c + 1) out[c] = 1;
        else if (nx + gr->w == c) out[c] = 2;
        else out[c] = 3;
    }
    return 0;
}

int orc_bfs_u16(orc_graph *gr, uint32_t goal, uint16_t *out) {
    if (goal >= gr->ncell || !gr->free_[goal]) return -1;
    for (uint32_t c = 0; c < gr->ncell; c++) out[c] = 0xFFFF;
    uint32_t *q = (uint32_t *)malloc(sizeof(uint32_t) * gr->ncell);
    size_t qh = 0, qt = 0;
    out[goal] = 0;
    q[qt++] = goal;
    while (qh < qt) {
        uint32_t c = q[qh++];
        for (uint32_t k = 0; k < gr->nbn[c]; k++) {
            uint32_t nc = gr->nb[4 * c + k];
            if (out[nc] == 0xFFFF) {
                out[nc] = (uint16_t)(out[c] + 1);
                q[qt++] = nc;
            }
        }
    }
    free(q);
    return 0;
}

/* agents.iter().position(|b| b.v == u) — lowest index, tswap.rs:192,223,269 */
static inline int64_t position_of(const uint32_t *v, uint32_t n, uint32_t u) {
    for (uint32_t k = 0; k < n; k++)
        if (v[k] == u) return k;
    return -1;
}

/* tswap_step, tswap.rs:174-286 */
int orc_tswap_step(orc_graph *gr, uint32_t *v, uint32_t *g, uint32_t n) {
    uint32_t *a_p = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    /* rules phase :180-252 */
    for (uint32_t i = 0; i < n; i++) {
        if (v[i] == g[i]) continue; /* rule 1 :182-184 */
        uint32_t u;
        int32_t len = orc_get_path_next(gr, v[i], g[i], &u, NULL);
        if (len < 2) continue;
        int64_t j = position_of(v, n, u);
        if (j < 0) continue;
        if ((uint32_t)j == i) continue;
        if (v[j] == g[j]) { /* rule 3 :198-202 */
            uint32_t gi = g[i], gj = g[j];
            g[i] = gj;
            g[j] = gi;
        } else { /* rule 4 :204-249 */
            size_t ap_len = 0;
            a_p[ap_len++] = i;
            uint32_t b = (uint32_t)j;
            int found = 0;
            for (;;) {
                uint32_t bv = v[b], bg = g[b];
                if (bv == bg) break;
                uint32_t w;
                int32_t bl = orc_get_path_next(gr, bv, bg, &w, NULL);
                if (bl < 2) break;
                int64_t c = position_of(v, n, w);
                if (c < 0) break;
                int contains = 0;
                for (size_t k = 0; k < ap_len; k++)
                    if (a_p[k] == b) {
                        contains = 1;
                        break;
                    }
                if (contains) {
                    ap_len = 0;
                    break;
                }
                a_p[ap_len++] = b;
                b = (uint32_t)c;
                if (b == i) {
                    found = 1;
                    break;
                }
            }
            if (found && ap_len > 1) { /* :241-249 */
                uint32_t first = a_p[0];
                uint32_t last_goal = g[a_p[ap_len - 1]];
                for (size_t k = ap_len - 1; k >= 1; k--) g[a_p[k]] = g[a_p[k - 1]];
                g[first] = last_goal;
            }
        }
    }
    /* movement phase :257-285 */
    for (uint32_t i = 0; i < n; i++) {
        if (v[i] == g[i]) continue;
        uint32_t u;
        int32_t len = orc_get_path_next(gr, v[i], g[i], &u, NULL);
        if (len < 2) continue;
        int64_t j = position_of(v, n, u);
        if (j >= 0) {
            if ((uint32_t)j != i) {
                uint32_t wj;
                int32_t lj = orc_get_path_next(gr, v[j], g[j], &wj, NULL);
                if (lj >= 2 && wj == v[i]) { /* mutual swap :273-278 */
                    uint32_t t = v[i];
                    v[i] = v[j];
                    v[j] = t;
                }
            }
        } else {
            v[i] = u; /* rule 2 :281-283 */
        }
    }
    free(a_p);
    return 0;
}

enum { ST_IDLE = 0, ST_TO_PICKUP = 1, ST_TO_DELIVERY = 2 };
enum { AS_PICKING = 0, AS_CARRYING = 1, AS_DELIVERED = 2, AS_IDLE = 3 };

static int xy_to_cell(const orc_graph *gr, uint32_t x, uint32_t y, uint32_t *c) {
    if (x >= gr->w || y >= gr->h) return -1;
    uint32_t cc = y * gr->w + x;
    if (!gr->free_[cc]) return -1;
    *c = cc;
    return 0;
}

/* tswap_mapd, tswap.rs:39-172 */
int32_t orc_tswap_mapd(orc_graph *gr, const uint32_t *starts_xy, uint32_t n,
                       const uint32_t *tasks_xyxy, uint32_t m, uint32_t max_t,
                       uint64_t *rec_out, uint32_t *goal_out) {
    uint32_t *v = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    uint32_t *g = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    uint8_t *st = (uint8_t *)calloc(n + 1, 1);
    int64_t *task_of = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    uint8_t *used = (uint8_t *)calloc(m + 1, 1);
    uint32_t *pick = (uint32_t *)malloc(sizeof(uint32_t) * (m + 1));
    uint32_t *dlv = (uint32_t *)malloc(sizeof(uint32_t) * (m + 1));
    int32_t T = -1;
    /* pos2id lookups panic on blocked/off-grid points (:94,112,136) */
    for (uint32_t i = 0; i < n; i++) {
        if (xy_to_cell(gr, starts_xy[2 * i], starts_xy[2 * i + 1], &v[i])) goto out;
        g[i] = v[i]; /* :92-101 */
        st[i] = ST_IDLE;
        task_of[i] = -1;
    }
    /* task cells are looked up only when used: pickup at assignment (:136), delivery on reaching the
     * pickup (:112) — an off-grid/blocked one panics there, not before */
    for (uint32_t k = 0; k < m; k++) {
        if (xy_to_cell(gr, tasks_xyxy[4 * k], tasks_xyxy[4 * k + 1], &pick[k])) pick[k] = UINT32_MAX;
        if (xy_to_cell(gr, tasks_xyxy[4 * k + 2], tasks_xyxy[4 * k + 3], &dlv[k])) dlv[k] = UINT32_MAX;
    }
    uint32_t unused = m;
    uint32_t timestep = 0;
    const uint32_t stride = max_t + 1;
    for (;;) {
        /* state and task management :106-139 */
        for (uint32_t i = 0; i < n; i++) {
            if (v[i] == g[i]) {
                if (st[i] == ST_TO_PICKUP) {
                    st[i] = ST_TO_DELIVERY;
                    if (task_of[i] >= 0) {
                        if (dlv[task_of[i]] == UINT32_MAX) goto out; /* pos2id[&task.delivery] panics */
                        g[i] = dlv[task_of[i]];
                    }
                } else if (st[i] == ST_TO_DELIVERY) {
                    st[i] = ST_IDLE;
                    task_of[i] = -1;
                }
            }
            if (st[i] == ST_IDLE && unused > 0) {
                /* min_by_key over unused tasks: first minimum wins (:125-130) */
                long px = v[i] % gr->w, py = v[i] / gr->w;
                int64_t best = -1;
                uint64_t bestd = 0;
                for (uint32_t k = 0; k < m; k++) {
                    if (used[k]) continue;
                    long dx = px - (long)tasks_xyxy[4 * k], dy = py - (long)tasks_xyxy[4 * k + 1];
                    uint64_t d = (uint64_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
                    if (best < 0 || d < bestd) {
                        best = k;
                        bestd = d;
                    }
                }
                if (best >= 0) {
                    used[best] = 1;
                    unused--;
                    task_of[i] = best;
                    st[i] = ST_TO_PICKUP;
                    if (pick[best] == UINT32_MAX) goto out; /* pos2id[&task.pickup] panics */
                    g[i] = pick[best];
                }
            }
        }
        orc_tswap_step(gr, v, g, n); /* :141 */
        /* record :144-158 */
        for (uint32_t i = 0; i < n; i++) {
            uint64_t s;
            if (st[i] == ST_IDLE) s = AS_IDLE;
            else if (st[i] == ST_TO_PICKUP) s = AS_PICKING;
            else s = (v[i] == g[i]) ? AS_DELIVERED : AS_CARRYING;
            uint64_t x = v[i] % gr->w, y = v[i] / gr->w;
            rec_out[(size_t)i * stride + timestep] = x | (y << 16) | (s << 32);
            if (goal_out) goal_out[(size_t)i * stride + timestep] = g[i];
        }
        timestep++;
        /* termination :163-169 */
        int all_idle = 1;
        for (uint32_t i = 0; i < n; i++)
            if (st[i] != ST_IDLE) {
                all_idle = 0;
                break;
            }
        if ((unused == 0 && all_idle) || timestep > max_t) break;
    }
    T = (int32_t)timestep;
out:
    free(v);
    free(g);
    free(st);
    free(task_of);
    free(used);
    free(pick);
    free(dlv);
    return T;
}

/* ---- decentralized decision --------------------------------------
 * compute_next_move_with_tswap, src/bin/decentralized/agent.rs:329-462, for one agent.
 * The local view is the caller's nearby list (agent.rs:108-153: every other agent within
 * Manhattan radius, self excluded) in the caller's order — `find` takes the FIRST entry at a
 * position (:369, :399-401, :435). Positions are cell ids; a position that is not a free cell
 * is "not in pos2id" (:392-393 break). */
static inline int64_t first_at(const uint32_t *nv, uint32_t nn, uint32_t pos) {
    for (uint32_t k = 0; k < nn; k++)
        if (nv[k] == pos) return k;
    return -1;
}

int orc_decide(orc_graph *gr, uint32_t my_v, uint32_t my_g, const uint32_t *nb_v, const uint32_t *nb_g,
               uint32_t nn, uint32_t *act, uint32_t *cell, uint32_t *partner, uint32_t *npart, uint32_t *part) {
    if (my_v >= gr->ncell || my_g >= gr->ncell || !gr->free_[my_v] || !gr->free_[my_g]) return -1; /* :358 panics */
    *cell = my_v;
    *partner = UINT32_MAX;
    *npart = 0;
    if (my_v == my_g) { /* Rule 1 :355-356 */
        *act = ORC_ACT_MOVE;
        return 0;
    }
    uint32_t next;
    int32_t len = orc_get_path_next(gr, my_v, my_g, &next, NULL); /* :358 */
    if (len < 2) { /* :359-360 */
        *act = ORC_ACT_MOVE;
        return 0;
    }
    int64_t b = first_at(nb_v, nn, next); /* :369 */
    if (b < 0) { /* Rule 2 :454-456 */
        *act = ORC_ACT_MOVE;
        *cell = next;
        return 0;
    }
    if (nb_v[b] == nb_g[b]) { /* Rule 3 :371-377 */
        *act = ORC_ACT_GOAL_SWAP;
        *partner = (uint32_t)b;
        return 0;
    }
    /* Rule 4 :379-427 — a_p holds POSITIONS */
    uint32_t *a_p = (uint32_t *)malloc(sizeof(uint32_t) * (nn + 2));
    size_t ap_len = 0;
    a_p[ap_len++] = my_v;
    uint32_t cur = (uint32_t)b;
    int found = 0;
    for (;;) {
        if (nb_v[cur] == nb_g[cur]) break; /* :383-385 */
        const uint32_t cv = nb_v[cur], cg = nb_g[cur];
        if (cv >= gr->ncell || !gr->free_[cv] || cg >= gr->ncell || !gr->free_[cg]) break; /* :389-393 */
        uint32_t nd;
        if (orc_get_path_next(gr, cv, cg, &nd, NULL) < 2) break; /* :393-397 */
        int64_t nx = first_at(nb_v, nn, nd); /* :399-401 */
        if (nx < 0) break; /* :416-419 */
        int in_ap = 0;
        for (size_t k = 0; k < ap_len; k++)
            if (a_p[k] == nb_v[nx]) in_ap = 1;
        if (in_ap) { /* :403-411 */
            if (nb_v[nx] == my_v) found = 1;
            else ap_len = 0;
            break;
        }
        a_p[ap_len++] = cv; /* :413 */
        cur = (uint32_t)nx;
    }
    if (found && ap_len > 1) { /* :430-447 */
        uint32_t np = 0;
        for (size_t k = 0; k < ap_len; k++) {
            int64_t a = first_at(nb_v, nn, a_p[k]);
            if (a >= 0) part[np++] = (uint32_t)a;
        }
        *npart = np;
        *act = np > 1 ? ORC_ACT_ROTATION : ORC_ACT_WAIT;
        if (np <= 1) *npart = 0;
    } else { /* Rule 5 :449-451 */
        *act = ORC_ACT_WAIT;
    }
    free(a_p);
    return 0;
}
