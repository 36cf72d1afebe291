/*
 * spec_sweep.c -- CPU-only probe for choosing FPSPEC v1. Not product code, not the oracle.
 *
 * sw_hashes: parametrised anchor -> target pairing over a peak list in (t, k) order (zone, fan-out, targets per
 * target frame, pair or triplet records); sw_query: FPSPEC 7 voting over a (hash, track, t)-sorted posting array
 * with the per-(track, d) score either the vote count (v0) or the number of distinct query anchor frames.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t mix32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

/* pairs: targets t2 in [t1 + dt_min, t1 + dt_max], |k2 - k1| <= df_max, at most `tpf` per target frame (0 = no
   limit), first `fan` in peak order. triplet > 0: records (anchor, target g, target h) for g < h <= g + triplet,
   hashed by mix32 of (k1, k2, k3, dt2, dt3). */
int64_t sw_hashes(const int32_t *pt, const int32_t *pk, int64_t np, int dt_min, int dt_max, int df_max, int fan,
                  int triplet, int tpf, int apf, uint32_t *hash, uint32_t *t1, int64_t cap) {
    int64_t n = 0;
    int acc_t[64], acc_k[64];
    int64_t frame_first = 0;
    for (int64_t i = 0; i < np; ++i) {
        if (i == 0 || pt[i] != pt[i - 1]) frame_first = i;
        if (apf && i - frame_first >= apf) continue;
        int got = 0, last_t = -1, in_frame = 0;
        for (int64_t j = i + 1; j < np && got < fan; ++j) {
            int32_t dt = pt[j] - pt[i];
            if (dt < dt_min) continue;
            if (dt > dt_max) break;
            int32_t df = pk[j] - pk[i];
            if (df < -df_max || df > df_max) continue;
            if (pt[j] != last_t) { last_t = pt[j]; in_frame = 0; }
            if (tpf && in_frame >= tpf) continue;
            ++in_frame;
            acc_t[got] = dt;
            acc_k[got] = pk[j];
            ++got;
        }
        if (!triplet) {
            for (int g = 0; g < got; ++g) {
                if (n < cap) {
                    hash[n] = ((uint32_t)(pk[i] & 0x3FF) << 22) | ((uint32_t)(acc_k[g] & 0x3FF) << 12) |
                              ((uint32_t)acc_t[g] & 0xFFF);
                    t1[n] = (uint32_t)pt[i];
                }
                ++n;
            }
        } else {
            for (int g = 0; g + 1 < got; ++g)
                for (int h = g + 1; h < got && h <= g + triplet; ++h) {
                    if (n < cap) {
                        uint64_t key = ((uint64_t)(pk[i] & 0x3FF) << 40) | ((uint64_t)(acc_k[g] & 0x3FF) << 30) |
                                       ((uint64_t)(acc_k[h] & 0x3FF) << 20) | ((uint64_t)(acc_t[g] & 0x3FF) << 10) |
                                       (uint64_t)(acc_t[h] & 0x3FF);
                        hash[n] = mix32(key);
                        t1[n] = (uint32_t)pt[i];
                    }
                    ++n;
                }
        }
    }
    return n;
}

typedef struct { uint32_t hash, track, t; } sw_posting;
typedef struct { uint32_t track; int32_t d; int32_t tq; } sw_vote;
typedef struct { int32_t score; uint32_t track; int32_t d; } sw_row;

static int cmp_vote(const void *a, const void *b) {
    const sw_vote *x = (const sw_vote *)a, *y = (const sw_vote *)b;
    if (x->track != y->track) return x->track < y->track ? -1 : 1;
    if (x->d != y->d) return x->d < y->d ? -1 : 1;
    return (x->tq > y->tq) - (x->tq < y->tq);
}
static int cmp_row(const void *a, const void *b) {
    const sw_row *x = (const sw_row *)a, *y = (const sw_row *)b;
    if (x->score != y->score) return x->score > y->score ? -1 : 1;
    return (x->track > y->track) - (x->track < y->track);
}

/* mode 0: score = votes of the best d (FPSPEC 7); mode 1: distinct query anchor frames of the best d;
   mode 2: distinct frames, but d within +-dtol merged (votes of d-dtol..d+dtol) */
int64_t sw_query(const sw_posting *p, int64_t np, const uint32_t *qh, const uint32_t *qt, int64_t nq, int mode,
                 int32_t min_score, sw_row *rows, int64_t max_rows) {
    int64_t cap = 4096, nv = 0;
    sw_vote *v = (sw_vote *)malloc(sizeof(sw_vote) * cap);
    for (int64_t i = 0; i < nq; ++i) {
        int64_t lo = 0, hi = np;
        while (lo < hi) { int64_t mid = (lo + hi) / 2; if (p[mid].hash < qh[i]) lo = mid + 1; else hi = mid; }
        for (int64_t j = lo; j < np && p[j].hash == qh[i]; ++j) {
            if (nv == cap) { cap *= 2; v = (sw_vote *)realloc(v, sizeof(sw_vote) * cap); }
            v[nv].track = p[j].track;
            v[nv].d = (int32_t)p[j].t - (int32_t)qt[i];
            v[nv].tq = (int32_t)qt[i];
            ++nv;
        }
    }
    qsort(v, (size_t)nv, sizeof(sw_vote), cmp_vote);
    int64_t nr = 0, rcap = 256;
    sw_row *all = (sw_row *)malloc(sizeof(sw_row) * rcap);
    int64_t i = 0;
    while (i < nv) {
        uint32_t tr = v[i].track;
        sw_row best = {0, tr, 0};
        while (i < nv && v[i].track == tr) {
            int32_t d = v[i].d, cnt = 0, last = -1;
            while (i < nv && v[i].track == tr && v[i].d == d) {
                if (mode == 0 || v[i].tq != last) ++cnt;
                last = v[i].tq;
                ++i;
            }
            if (cnt > best.score) { best.score = cnt; best.d = d; }
        }
        if (best.score >= min_score) {
            if (nr == rcap) { rcap *= 2; all = (sw_row *)realloc(all, sizeof(sw_row) * rcap); }
            all[nr++] = best;
        }
    }
    qsort(all, (size_t)nr, sizeof(sw_row), cmp_row);
    if (nr > max_rows) nr = max_rows;
    memcpy(rows, all, sizeof(sw_row) * (size_t)nr);
    free(all);
    free(v);
    return nr;
}
