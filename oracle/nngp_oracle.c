/*
 * C restatement of the NNGP neighbour-set + B/F + log-likelihood path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker / timed CPU baseline.  The product
 * (pynngp_amd, libnngp_hip.so) never links or calls it.
 *
 * Reference (bwpriest/pyNNGP, /root/reference):
 *   oracle_knn_prior  <- NNGP._make_s_neighbor_sets, pyNNGP/nngp.py:49-62
 *                        (sklearn 1.7.2 KDTree.query, sort_results=True; key is
 *                         euclidean_rdist64, sklearn/metrics/_dist_metrics.pxd:26-40)
 *   oracle_bf_sweep   <- _CNs nngp.py:78-82, _Ccross :84-86, _Cs :92-96,
 *                        _Bsi :73-76, _Fsi :88-90 (stubs in the reference; NNGP
 *                        definitions of SURVEY.md Appendix A)
 * Same math as oracle/nngp_oracle.py; that file's header states the pinning.
 *
 * Compiled with -ffp-contract=off so rdist is (0 + t0*t0) + t1*t1 exactly as
 * sklearn's x86-64 build computes it (no FMA).  Ties: lower index first.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

static inline int key_less(double da, int64_t ia, double db, int64_t ib) {
    return da < db || (da == db && ia < ib);
}

/* sklearn euclidean_rdist64: d = 0; d += t_k * t_k for k = 0 .. dim-1 (no FMA: -ffp-contract=off) */
static inline double rdist(const double *a, const double *b, int dim) {
    double d = 0.0;
    for (int k = 0; k < dim; ++k) {
        const double t = a[k] - b[k];
        d += t * t;
    }
    return d;
}

/* nngp.py:49-62 -- brute force over j < i, kept sorted by (rdist, j); coords (n, dim). */
int oracle_knn_prior(const double *coords, int64_t n, int32_t dim, int32_t m, int64_t q0, int64_t q1, int32_t *nbr) {
    if (m < 0 || dim < 1 || q0 < 0 || q1 > n || q0 > q1) return -1;
    if (m == 0) return 0;
#pragma omp parallel
    {
        double *bd = (double *)malloc(sizeof(double) * (size_t)m);
        int64_t *bi = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = q0; i < q1; ++i) {
            int32_t *row = nbr + (i - q0) * m;
            int64_t k = i < m ? i : m;
            int64_t cnt = 0;
            const double *qi = coords + i * dim;
            for (int64_t j = 0; j < i; ++j) {
                const double d = rdist(qi, coords + j * dim, dim);
                if (cnt == k && !key_less(d, j, bd[k - 1], bi[k - 1])) continue;
                int64_t s = cnt < k ? cnt++ : k - 1;
                while (s > 0 && key_less(d, j, bd[s - 1], bi[s - 1])) {
                    bd[s] = bd[s - 1];
                    bi[s] = bi[s - 1];
                    --s;
                }
                bd[s] = d;
                bi[s] = j;
            }
            for (int64_t s = 0; s < m; ++s) row[s] = s < k ? (int32_t)bi[s] : -1;
        }
        free(bd);
        free(bi);
    }
    return 0;
}

/* Same sets for an explicit list of query rows (parallel over the list): row t of nbr is
 * the set of location rows[t].  Used for sampled-row checks at N = 1e7, where one call
 * per row would scan s[0:i] on a single thread. */
int oracle_knn_prior_rows(const double *coords, int64_t n, int32_t dim, int32_t m, const int64_t *rows,
                          int64_t n_rows, int32_t *nbr) {
    if (m < 0 || dim < 1 || n_rows < 0) return -1;
    for (int64_t t = 0; t < n_rows; ++t)
        if (rows[t] < 0 || rows[t] >= n) return -1;
    int rc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : rc)
    for (int64_t t = 0; t < n_rows; ++t) rc |= oracle_knn_prior(coords, n, dim, m, rows[t], rows[t] + 1, nbr + t * m);
    return rc;
}

/* Covariance kinds (the reference's `cov` plug-in, nngp.py:6,12), u = phi d:
 *   0 exponential sigma2 e^-u   1 matern32 sigma2 (1 + u) e^-u   2 matern52 sigma2 (1 + u + u^2/3) e^-u
 *   3 gaussian    sigma2 e^-u^2 4 spherical sigma2 (1 - 3u/2 + u^3/2) for u < 1, else 0
 *   5 matern      sigma2 u^nu K_nu(u) / (2^(nu-1) Gamma(nu)), nu = theta[3] (matern_rho below) */
/* ---------------------------------------------------------------------------
 * The reference's own neighbour-set ALGORITHM, restated for the CPU baseline:
 * NNGP._make_s_neighbor_sets (nngp.py:49-62) builds a fresh sklearn KDTree over
 * s[0:i] for every i (nngp.py:55) and queries the k = min(m, i) nearest
 * (nngp.py:56-61), O(N^2 log N) in all.  Same construction here, single thread (the
 * reference's loop is a single Python thread): per i, a kd-tree over s[0:i] with
 * sklearn's defaults (leaf_size 40, split on the dimension of largest spread at the
 * median, sklearn/neighbors/_kd_tree.pyx + _binary_tree.pxi.tp:1086-1195), then a
 * depth-first query with a bounded max-heap and node-box pruning
 * (_binary_tree.pxi.tp:1604-1658).  Keys are (rdist, index), so the result equals
 * oracle_knn_prior bit for bit (the box bound is a true lower bound of the fp rdist:
 * correctly rounded sub / mul / add are monotone).
 * ------------------------------------------------------------------------- */
typedef struct {
    int64_t start, end;  /* idx[start:end] */
    int64_t left, right; /* children, -1 for a leaf */
} KdNode;

typedef struct {
    const double *pts;
    int dim;
    int64_t *idx;
    KdNode *nodes;
    double *lo, *hi; /* node boxes, dim each */
    int64_t n_nodes;
} KdTree;

static void kd_swap(int64_t *a, int64_t *b) { int64_t t = *a; *a = *b; *b = t; }

/* place the median (by coordinate k) at idx[mid], smaller before, larger after (quickselect) */
static void kd_select(const double *pts, int dim, int k, int64_t *idx, int64_t lo, int64_t hi, int64_t mid) {
    while (hi - lo > 1) {
        const double pv = pts[idx[(lo + hi) / 2] * dim + k];
        int64_t a = lo, b = hi - 1;
        while (a <= b) {
            while (pts[idx[a] * dim + k] < pv) ++a;
            while (pts[idx[b] * dim + k] > pv) --b;
            if (a <= b) kd_swap(&idx[a++], &idx[b--]);
        }
        if (mid <= b) hi = b + 1;
        else if (mid >= a) lo = a;
        else return;
    }
}

static int64_t kd_build(KdTree *t, int64_t start, int64_t end) {
    const int64_t id = t->n_nodes++;
    KdNode *nd = &t->nodes[id];
    nd->start = start;
    nd->end = end;
    nd->left = nd->right = -1;
    double *lo = t->lo + id * t->dim, *hi = t->hi + id * t->dim;
    for (int k = 0; k < t->dim; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
    }
    for (int64_t a = start; a < end; ++a)
        for (int k = 0; k < t->dim; ++k) {
            const double v = t->pts[t->idx[a] * t->dim + k];
            if (v < lo[k]) lo[k] = v;
            if (v > hi[k]) hi[k] = v;
        }
    if (end - start <= 40) return id; /* sklearn's default leaf_size */
    int ks = 0;
    for (int k = 1; k < t->dim; ++k)
        if (hi[k] - lo[k] > hi[ks] - lo[ks]) ks = k;
    const int64_t mid = start + (end - start) / 2;
    kd_select(t->pts, t->dim, ks, t->idx, start, end, mid);
    const int64_t l = kd_build(t, start, mid);
    const int64_t r = kd_build(t, mid, end);
    t->nodes[id].left = l;
    t->nodes[id].right = r;
    return id;
}

static double kd_min_rdist(const KdTree *t, int64_t id, const double *q) {
    const double *lo = t->lo + id * t->dim, *hi = t->hi + id * t->dim;
    double d = 0.0;
    for (int k = 0; k < t->dim; ++k) {
        double e = 0.0;
        if (q[k] < lo[k]) e = lo[k] - q[k];
        else if (q[k] > hi[k]) e = q[k] - hi[k];
        d += e * e;
    }
    return d;
}

/* bounded sorted list of the k best (rdist, j) */
static void kd_push(double *bd, int64_t *bi, int64_t *cnt, int64_t k, double d, int64_t j) {
    if (*cnt == k && !key_less(d, j, bd[k - 1], bi[k - 1])) return;
    int64_t s = *cnt < k ? (*cnt)++ : k - 1;
    while (s > 0 && key_less(d, j, bd[s - 1], bi[s - 1])) {
        bd[s] = bd[s - 1];
        bi[s] = bi[s - 1];
        --s;
    }
    bd[s] = d;
    bi[s] = j;
}

static void kd_query(const KdTree *t, int64_t id, const double *q, int64_t k, double *bd, int64_t *bi, int64_t *cnt) {
    const KdNode *nd = &t->nodes[id];
    if (*cnt == k && kd_min_rdist(t, id, q) > bd[k - 1]) return;
    if (nd->left < 0) {
        for (int64_t a = nd->start; a < nd->end; ++a) {
            const int64_t j = t->idx[a];
            kd_push(bd, bi, cnt, k, rdist(q, t->pts + j * t->dim, t->dim), j);
        }
        return;
    }
    const double dl = kd_min_rdist(t, nd->left, q), dr = kd_min_rdist(t, nd->right, q);
    const int64_t first = dl <= dr ? nd->left : nd->right, second = dl <= dr ? nd->right : nd->left;
    kd_query(t, first, q, k, bd, bi, cnt);
    kd_query(t, second, q, k, bd, bi, cnt);
}

int oracle_knn_prior_kdtree_rebuild(const double *coords, int64_t n, int32_t dim, int32_t m, int64_t q0, int64_t q1,
                                    int32_t *nbr) {
    if (m < 0 || dim < 1 || q0 < 0 || q1 > n || q0 > q1) return -1;
    if (m == 0 || q1 == q0) return 0;
    const int64_t cap = q1 > 1 ? q1 : 1;
    KdTree t;
    t.pts = coords;
    t.dim = dim;
    t.idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    t.nodes = (KdNode *)malloc(sizeof(KdNode) * (size_t)(2 * cap / 20 + 8));
    t.lo = (double *)malloc(sizeof(double) * (size_t)dim * (size_t)(2 * cap / 20 + 8));
    t.hi = (double *)malloc(sizeof(double) * (size_t)dim * (size_t)(2 * cap / 20 + 8));
    double *bd = (double *)malloc(sizeof(double) * (size_t)m);
    int64_t *bi = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
    for (int64_t i = q0; i < q1; ++i) {
        int32_t *row = nbr + (i - q0) * m;
        const int64_t k = i < m ? i : m;
        int64_t cnt = 0;
        if (i > 0) {
            for (int64_t a = 0; a < i; ++a) t.idx[a] = a; /* KDTree(s[0:i]): a fresh tree per i */
            t.n_nodes = 0;
            kd_build(&t, 0, i);
            kd_query(&t, 0, coords + i * dim, k, bd, bi, &cnt);
        }
        for (int64_t s = 0; s < m; ++s) row[s] = s < cnt ? (int32_t)bi[s] : -1;
    }
    free(t.idx);
    free(t.nodes);
    free(t.lo);
    free(t.hi);
    free(bd);
    free(bi);
    return 0;
}

/* ---------------------------------------------------------------------------
 * An exact prior-kNN for large N that shares nothing with the GPU's grid search
 * (pynngp_amd/csrc/knn.hip): kd-trees over DOUBLING PREFIXES s[0:2^k].  Query i
 * searches the tree of the smallest prefix that holds s[0:i] (2^k >= i, so at least
 * half of that tree's points are prior points) and skips every j >= i.  Same key as
 * nngp.py:49-62 through sklearn (rdist unfused, ascending; ties by lower index, the
 * documented divergence), same kd-tree code as the per-i rebuild above; the node-box
 * bound prunes only with '>' so keys tied with the k-th are still visited.  The trees
 * total ~2N points (O(N log N) to build instead of the reference's O(N^2 log N)), so
 * every row of config 4 (N = 1e7, m = 20) is checkable in seconds.
 * ------------------------------------------------------------------------- */
static void kd_query_prior(const KdTree *t, int64_t id, const double *q, int64_t i, int64_t k, double *bd,
                           int64_t *bi, int64_t *cnt) {
    const KdNode *nd = &t->nodes[id];
    if (*cnt == k && kd_min_rdist(t, id, q) > bd[k - 1]) return;
    if (nd->left < 0) {
        for (int64_t a = nd->start; a < nd->end; ++a) {
            const int64_t j = t->idx[a];
            if (j < i) kd_push(bd, bi, cnt, k, rdist(q, t->pts + j * t->dim, t->dim), j);
        }
        return;
    }
    const double dl = kd_min_rdist(t, nd->left, q), dr = kd_min_rdist(t, nd->right, q);
    const int64_t first = dl <= dr ? nd->left : nd->right, second = dl <= dr ? nd->right : nd->left;
    kd_query_prior(t, first, q, i, k, bd, bi, cnt);
    kd_query_prior(t, second, q, i, k, bd, bi, cnt);
}

static int kd_alloc(KdTree *t, const double *pts, int dim, int64_t size) {
    const int64_t nn = 2 * size / 20 + 8;
    t->pts = pts;
    t->dim = dim;
    t->n_nodes = 0;
    t->idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)(size > 0 ? size : 1));
    t->nodes = (KdNode *)malloc(sizeof(KdNode) * (size_t)nn);
    t->lo = (double *)malloc(sizeof(double) * (size_t)dim * (size_t)nn);
    t->hi = (double *)malloc(sizeof(double) * (size_t)dim * (size_t)nn);
    return t->idx && t->nodes && t->lo && t->hi;
}

static void kd_free(KdTree *t) {
    free(t->idx);
    free(t->nodes);
    free(t->lo);
    free(t->hi);
}

static int64_t kd_size(int k, int64_t n) { return ((int64_t)1 << k) > n ? n : ((int64_t)1 << k); }

/* smallest k with 2^k >= i (i >= 1) */
static int ceil_log2(int64_t i) {
    int k = 0;
    while (((int64_t)1 << k) < i) ++k;
    return k;
}

/* nodes of the kd_build subtree over `size` points (sizes at one depth are floor / ceil of
 * one value, so the pair (c(a), c(a+1)) recurses on a / 2 alone) */
static void kd_count_pair(int64_t a, int64_t *ca, int64_t *ca1) {
    if (a + 1 <= 40) {
        *ca = 1;
        *ca1 = 1;
        return;
    }
    if (a <= 40) { /* a = 40: c(41) = 1 + c(20) + c(21) */
        *ca = 1;
        *ca1 = 3;
        return;
    }
    int64_t ch, ch1;
    kd_count_pair(a / 2, &ch, &ch1);
    if (a % 2 == 0) {
        *ca = 1 + 2 * ch;
        *ca1 = 1 + ch + ch1;
    } else {
        *ca = 1 + ch + ch1;
        *ca1 = 1 + 2 * ch1;
    }
}

static int64_t kd_count(int64_t size) {
    int64_t c, c1;
    kd_count_pair(size, &c, &c1);
    return c;
}

/* kd_build with the same tree and node numbering (pre-order: left child id + 1, right child
 * id + 1 + nodes of the left subtree), subtrees of large nodes built as OpenMP tasks */
static void kd_build_at(KdTree *t, int64_t id, int64_t start, int64_t end) {
    KdNode *nd = &t->nodes[id];
    nd->start = start;
    nd->end = end;
    nd->left = nd->right = -1;
    double *lo = t->lo + id * t->dim, *hi = t->hi + id * t->dim;
    for (int k = 0; k < t->dim; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
    }
    for (int64_t a = start; a < end; ++a)
        for (int k = 0; k < t->dim; ++k) {
            const double v = t->pts[t->idx[a] * t->dim + k];
            if (v < lo[k]) lo[k] = v;
            if (v > hi[k]) hi[k] = v;
        }
    if (end - start <= 40) return;
    int ks = 0;
    for (int k = 1; k < t->dim; ++k)
        if (hi[k] - lo[k] > hi[ks] - lo[ks]) ks = k;
    const int64_t mid = start + (end - start) / 2;
    kd_select(t->pts, t->dim, ks, t->idx, start, end, mid);
    const int64_t l = id + 1, r = id + 1 + kd_count(mid - start);
    nd->left = l;
    nd->right = r;
    if (end - start > 65536) {
#pragma omp task
        kd_build_at(t, l, start, mid);
#pragma omp task
        kd_build_at(t, r, mid, end);
#pragma omp taskwait
    } else {
        kd_build_at(t, l, start, mid);
        kd_build_at(t, r, mid, end);
    }
}

static void knn_prior_row(const KdTree *t, const double *coords, int dim, int64_t i, int32_t m, double *bd,
                          int64_t *bi, int32_t *row) {
    const int64_t k = i < m ? i : m;
    int64_t cnt = 0;
    kd_query_prior(t, 0, coords + i * dim, i, k, bd, bi, &cnt);
    for (int64_t s = 0; s < m; ++s) row[s] = s < cnt ? (int32_t)bi[s] : -1;
}

int oracle_knn_prior_prefix_kdtree(const double *coords, int64_t n, int32_t dim, int32_t m, int64_t q0, int64_t q1,
                                   int32_t *nbr) {
    if (m < 0 || dim < 1 || q0 < 0 || q1 > n || q0 > q1) return -1;
    if (m == 0 || q1 == q0) return 0;
    const int64_t first = q0 > 1 ? q0 : 1; /* row 0 has no prior point */
    const int klo = ceil_log2(first), khi = q1 - 1 >= first ? ceil_log2(q1 - 1) : klo;
    const int nlev = khi - klo + 1;
    KdTree *trees = (KdTree *)calloc((size_t)nlev, sizeof(KdTree));
    if (trees == NULL) return -2;
    int rc = 0;
    for (int l = 0; l < nlev; ++l) {
        if (!kd_alloc(&trees[l], coords, dim, kd_size(klo + l, n))) rc = 1;
    }
    /* one task tree per prefix, the large nodes' subtrees as tasks of their own */
#pragma omp parallel
#pragma omp single
    for (int l = nlev - 1; l >= 0 && rc == 0; --l) {
#pragma omp task firstprivate(l)
        {
            KdTree *t = &trees[l];
            const int64_t size = kd_size(klo + l, n);
            for (int64_t a = 0; a < size; ++a) t->idx[a] = a;
            kd_build_at(t, 0, 0, size);
            t->n_nodes = kd_count(size);
        }
    }
    if (rc == 0) {
#pragma omp parallel
        {
            double *bd = (double *)malloc(sizeof(double) * (size_t)m);
            int64_t *bi = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
            /* query i (not a power of two) is a point of the tree it searches: visiting the
             * queries in that tree's leaf order (spatial order) keeps consecutive queries on the
             * same paths and leaves.  i = 2^k searches tree k without being one of its points,
             * and row 0 has no prior point: both are done on their own. */
            for (int l = 0; l < nlev; ++l) {
                const KdTree *t = &trees[l];
                const int64_t size = kd_size(klo + l, n);
#pragma omp for schedule(dynamic, 256) nowait
                for (int64_t a = 0; a < size; ++a) {
                    const int64_t i = t->idx[a];
                    if (i < q0 || i >= q1 || i < 1 || (i & (i - 1)) == 0 || ceil_log2(i) != klo + l) continue;
                    knn_prior_row(t, coords, dim, i, m, bd, bi, nbr + (i - q0) * m);
                }
            }
#pragma omp for schedule(dynamic, 1)
            for (int k = 0; k < 63; ++k) {
                const int64_t i = (int64_t)1 << k;
                if (i >= q0 && i < q1) knn_prior_row(&trees[k - klo], coords, dim, i, m, bd, bi, nbr + (i - q0) * m);
            }
#pragma omp single
            if (q0 == 0)
                for (int64_t s = 0; s < m; ++s) nbr[s] = -1;
            free(bd);
            free(bi);
        }
    }
    for (int l = 0; l < nlev; ++l) kd_free(&trees[l]);
    free(trees);
    return rc ? -2 : 0;
}

/* Matern of general smoothness nu (kind 5, spNNGP's "matern"): rho(u) = u^nu K_nu(u) / (2^(nu-1) Gamma(nu))
 * from the integral K_nu(u) = int_0^inf exp(-u cosh t) cosh(nu t) dt (Watson 6.22 (5)) by the trapezoidal
 * rule in long double -- a method independent of the kernels' Temme series / continued fraction
 * (nngp_math.h).  The integrand is entire and decays double-exponentially, so the trapezoidal error is
 * ~exp(-2 pi a / h) times the integrand's growth into the strip |Im t| < a, ~(cos a)^-nu: h = 1/20
 * leaves < 1e-25 up to nu = 50; for large u the integrand is a peak of width ~u^-1/2 at t = 0, so
 * h <= u^-1/2 / 4 (the Gaussian's trapezoidal error ~exp(-2 pi^2 / (16 h^2 u)) ~ 1e-53).  Every term is summed as
 * exp(log term): nu ln u - u cosh t + ln cosh(nu t) - ln(2^(nu-1) Gamma(nu)), so nothing over- or
 * underflows for any u > 0 (u^nu and K_nu(u) separately would for tiny u). */
static double matern_rho(double nu, double u) {
    if (!(u > 0.0)) return 1.0;
    const long double hw = 0.25L / sqrtl((long double)u);
    const long double h = hw < 0.05L ? hw : 0.05L, lu = logl((long double)u), nul = (long double)nu;
    const long double lnorm = (nul - 1.0L) * logl(2.0L) + lgammal(nul);
    const long double tpk = asinhl(nul / (long double)u); /* the integrand's peak */
    long double sum = 0.0L, emax = -INFINITY;
    for (long k = 0;; ++k) {
        const long double t = h * (long double)k;
        const long double lch = nul * t + log1pl(expl(-2.0L * nul * t)) - logl(2.0L); /* ln cosh(nu t) */
        const long double e = nul * lu - (long double)u * coshl(t) + lch - lnorm;
        if (e > emax) emax = e;
        sum += (k == 0 ? 0.5L : 1.0L) * expl(e);
        if (t > tpk && e < emax - 100.0L) break;
    }
    return (double)(h * sum);
}

static inline double cov_eval_nu(int kind, double d, double sigma2, double phi, double nu) {
    const double u = phi * d;
    switch (kind) {
        case 5: return sigma2 * matern_rho(nu, u);
        case 1: return sigma2 * (1.0 + u) * exp(-u);
        case 2: return sigma2 * (1.0 + u + u * u / 3.0) * exp(-u);
        case 3: return sigma2 * exp(-u * u);
        case 4: return u < 1.0 ? sigma2 * (1.0 - 1.5 * u + 0.5 * u * u * u) : 0.0;
        default: return sigma2 * exp(-u);
    }
}

/* exported for tests/test_matern.py (the restatement checked against mpmath) */
double oracle_matern_rho(double nu, double u) { return matern_rho(nu, u); }

static inline double pdist(const double *a, const double *b, int dim) { return sqrt(rdist(a, b, dim)); }

/*
 * Per location: C_N (+tau2 I), c, C_ii -> Cholesky C_N = L L^T (row-oriented),
 * v = L^-1 c, B = L^-T v, F = C_ii - v.v, r = v_i - B.v_N.
 * partials[0] = sum log F, partials[1] = sum r^2/F (index order),
 * partials[2] = first row index whose pivot or F is not > 0 (or -1).
 * A slot is valid iff its index is >= 0; -1 slots give B = 0; an index >= n or below -1
 * marks the row bad (B = F = NaN, partials[2]).
 */
int oracle_bf_sweep(const double *coords, const int32_t *nbr, int64_t n, int32_t dim, int32_t m, int32_t kind,
                    const double *theta, const double *values, double *Bout, double *Fout, double *partials,
                    int64_t i0, int64_t i1) {
    if (m < 0 || dim < 1 || i0 < 0 || i1 > n || i0 > i1 || kind < 0 || kind > 5) return -1;
    const double sigma2 = theta[0], phi = theta[1], tau2 = theta[2];
    const double nu = kind == 5 ? theta[3] : 0.0; /* theta = (sigma2, phi, tau2, nu) for kind 5 */
    const int64_t rows = i1 - i0;
    double *logF = (double *)malloc(sizeof(double) * (size_t)(rows > 0 ? rows : 1));
    double *quad = (double *)malloc(sizeof(double) * (size_t)(rows > 0 ? rows : 1));
    int64_t first_bad = INT64_MAX;
#pragma omp parallel
    {
        const int mm = m > 0 ? m : 1;
        double *L = (double *)malloc(sizeof(double) * (size_t)mm * mm);
        double *c = (double *)malloc(sizeof(double) * (size_t)mm);
        double *v = (double *)malloc(sizeof(double) * (size_t)mm);
        double *b = (double *)malloc(sizeof(double) * (size_t)mm);
        int *slot = (int *)malloc(sizeof(int) * (size_t)mm);
        int64_t bad_local = INT64_MAX;
#pragma omp for schedule(static)
        for (int64_t r = 0; r < rows; ++r) {
            const int64_t i = i0 + r;
            const int32_t *row = nbr + r * m;
            int k = 0;
            int bad = 0;
            for (int s = 0; s < m; ++s)
                if (row[s] >= 0) {
                    if (row[s] >= n) bad = 1;
                    slot[k++] = s;
                } else if (row[s] != -1) {
                    bad = 1; /* only -1 pads a row */
                }
            const double *xi = coords + dim * i;
            double F = sigma2 + tau2;
            double rr = bad ? NAN : (values ? values[i] : 0.0);
            if (!bad) {
                for (int a = 0; a < k; ++a) {
                    const double *xa = coords + dim * (int64_t)row[slot[a]];
                    for (int bb = 0; bb < a; ++bb) {
                        const double *xb = coords + dim * (int64_t)row[slot[bb]];
                        L[a * k + bb] = cov_eval_nu(kind, pdist(xa, xb, dim), sigma2, phi, nu);
                    }
                    L[a * k + a] = sigma2 + tau2;
                    c[a] = cov_eval_nu(kind, pdist(xi, xa, dim), sigma2, phi, nu);
                }
                /* Cholesky (Cholesky-Banachiewicz, row by row) */
                for (int a = 0; a < k && !bad; ++a) {
                    for (int bb = 0; bb <= a; ++bb) {
                        double s = L[a * k + bb];
                        for (int q = 0; q < bb; ++q) s -= L[a * k + q] * L[bb * k + q];
                        if (bb == a) {
                            if (!(s > 0.0)) { bad = 1; break; }
                            L[a * k + a] = sqrt(s);
                        } else {
                            L[a * k + bb] = s / L[bb * k + bb];
                        }
                    }
                }
            }
            if (!bad) {
                for (int a = 0; a < k; ++a) { /* v = L^-1 c */
                    double s = c[a];
                    for (int q = 0; q < a; ++q) s -= L[a * k + q] * v[q];
                    v[a] = s / L[a * k + a];
                }
                for (int a = k - 1; a >= 0; --a) { /* B = L^-T v */
                    double s = v[a];
                    for (int q = a + 1; q < k; ++q) s -= L[q * k + a] * b[q];
                    b[a] = s / L[a * k + a];
                }
                double vv = 0.0, bv = 0.0;
                for (int a = 0; a < k; ++a) vv += v[a] * v[a];
                F = (sigma2 + tau2) - vv;
                if (values)
                    for (int a = 0; a < k; ++a) bv += b[a] * values[row[slot[a]]];
                rr = values ? values[i] - bv : 0.0;
                if (!(F > 0.0)) bad = 1;
            }
            if (Bout) {
                double *brow = Bout + r * m;
                for (int s = 0; s < m; ++s) brow[s] = 0.0;
                for (int a = 0; a < k; ++a) brow[slot[a]] = bad ? NAN : b[a];
            }
            if (bad) {
                F = NAN;
                if (i < bad_local) bad_local = i;
            }
            if (Fout) Fout[r] = F;
            logF[r] = log(F);
            quad[r] = rr * rr / F;
        }
#pragma omp critical
        if (bad_local < first_bad) first_bad = bad_local;
        free(L);
        free(c);
        free(v);
        free(b);
        free(slot);
    }
    double s0 = 0.0, s1 = 0.0;
    for (int64_t r = 0; r < rows; ++r) {
        s0 += logF[r];
        s1 += quad[r];
    }
    partials[0] = s0;
    partials[1] = s1;
    partials[2] = first_bad == INT64_MAX ? -1.0 : (double)first_bad;
    free(logF);
    free(quad);
    return 0;
}

/* Draw w ~ NNGP(0, C~) by forward substitution through the DAG the neighbour sets
 * define: w_i = sum_k B_ik w_{N(i)_k} + sqrt(F_i) eps_i, in location order (every
 * neighbour of i precedes i).  This is the density the B/F sweep evaluates
 * (the factorisation behind _Bsi/_Fsi nngp.py:73-90); the
 * reference has no simulator.  Used by the tests to draw large fields whose law is
 * exactly the NNGP (a dense GP draw is out of reach at N = 1e6). */
int oracle_nngp_simulate(const int32_t *nbr, const double *B, const double *F, int64_t n, int32_t m,
                         const double *eps, double *w) {
    for (int64_t i = 0; i < n; ++i) {
        double acc = 0.0;
        for (int32_t k = 0; k < m; ++k) {
            int32_t j = nbr[i * m + k];
            if (j < 0) continue;
            if (j >= i) return -1;
            acc += B[i * m + k] * w[j];
        }
        if (!(F[i] > 0.0)) return -2;
        w[i] = acc + sqrt(F[i]) * eps[i];
    }
    return 0;
}
