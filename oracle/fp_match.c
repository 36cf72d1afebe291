/*
 * fp_match.c -- CPU restatement of spec/FPSPEC.md section 7 (index + query), FPSPEC v1: a (track, d)
 * scores the distinct query anchor frames that vote for it (v0 counted the votes themselves).
 * TEST INFRASTRUCTURE ONLY (see fp_oracle.c header): it checks the GPU
 * index/match kernels; it is never the product path.
 *
 * Replaces (as a checker) what `olaf_c store` / `olaf_c query` do behind
 * audio-ident-service/app/audio/fingerprint.py:117-125 and :185-202: an inverted
 * index keyed by hash, and per-track offset voting whose best bin becomes
 * OlafMatch.match_count (fingerprint.py:44-50).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint32_t hash, track, t; } fp_posting;
typedef struct { int32_t match_count; uint32_t track; int32_t d; int32_t tq_min, tq_max; } fp_row;
typedef struct { uint32_t track; int32_t d; int32_t tq; } vote;

static int cmp_posting(const void *a, const void *b) {
    const fp_posting *x = (const fp_posting *)a, *y = (const fp_posting *)b;
    if (x->hash != y->hash) return x->hash < y->hash ? -1 : 1;
    if (x->track != y->track) return x->track < y->track ? -1 : 1;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    return 0;
}

static int cmp_vote(const void *a, const void *b) {
    const vote *x = (const vote *)a, *y = (const vote *)b;
    if (x->track != y->track) return x->track < y->track ? -1 : 1;
    if (x->d != y->d) return x->d < y->d ? -1 : 1;
    if (x->tq != y->tq) return x->tq < y->tq ? -1 : 1;
    return 0;
}

static int cmp_row(const void *a, const void *b) {
    const fp_row *x = (const fp_row *)a, *y = (const fp_row *)b;
    if (x->match_count != y->match_count) return x->match_count > y->match_count ? -1 : 1;
    return x->track < y->track ? -1 : (x->track > y->track);
}

/* sorts postings in place by (hash, track, t) */
void fp_index_sort(fp_posting *p, int64_t n) { qsort(p, (size_t)n, sizeof(fp_posting), cmp_posting); }

static int64_t lower_bound(const fp_posting *p, int64_t n, uint32_t h) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (p[mid].hash < h) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* postings must be sorted (fp_index_sort). Returns rows written (<= max_rows). */
int64_t fp_query(const fp_posting *p, int64_t np, const uint32_t *qhash, const uint32_t *qt, int64_t nq,
                 int32_t min_match, fp_row *rows, int64_t max_rows) {
    int64_t cap = 1024, nv = 0;
    vote *v = (vote *)malloc(sizeof(vote) * cap);
    for (int64_t i = 0; i < nq; ++i) {
        for (int64_t j = lower_bound(p, np, qhash[i]); j < np && p[j].hash == qhash[i]; ++j) {
            if (nv == cap) { cap *= 2; v = (vote *)realloc(v, sizeof(vote) * cap); }
            v[nv].track = p[j].track;
            v[nv].d = (int32_t)p[j].t - (int32_t)qt[i];
            v[nv].tq = (int32_t)qt[i];
            ++nv;
        }
    }
    qsort(v, (size_t)nv, sizeof(vote), cmp_vote);
    int64_t nr = 0, rcap = 256;
    fp_row *all = (fp_row *)malloc(sizeof(fp_row) * rcap);
    int64_t i = 0;
    while (i < nv) {
        uint32_t tr = v[i].track;
        fp_row best = {0, tr, 0, 0, 0};
        while (i < nv && v[i].track == tr) {
            /* FPSPEC v1 7: the score of (track, d) is the number of DISTINCT query anchor frames t_q among its
               votes (votes are sorted by (track, d, t_q), so a new t_q is a change from the previous vote) */
            int32_t d = v[i].d, cnt = 0, lo = v[i].tq, hi = v[i].tq, last = 0;
            int first = 1;
            while (i < nv && v[i].track == tr && v[i].d == d) {
                if (v[i].tq < lo) lo = v[i].tq;
                if (v[i].tq > hi) hi = v[i].tq;
                if (first || v[i].tq != last) ++cnt;
                last = v[i].tq;
                first = 0;
                ++i;
            }
            if (cnt > best.match_count) { best.match_count = cnt; best.d = d; best.tq_min = lo; best.tq_max = hi; }
        }
        if (best.match_count >= min_match) {
            if (nr == rcap) { rcap *= 2; all = (fp_row *)realloc(all, sizeof(fp_row) * rcap); }
            all[nr++] = best;
        }
    }
    qsort(all, (size_t)nr, sizeof(fp_row), cmp_row);
    if (nr > max_rows) nr = max_rows;
    memcpy(rows, all, sizeof(fp_row) * (size_t)nr);
    free(all);
    free(v);
    return nr;
}
