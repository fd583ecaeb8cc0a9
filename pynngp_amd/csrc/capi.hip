// C ABI of libnngp_hip.so (declared in include/nngp.h): argument checking,
// workspace carving and launch.  No host synchronisation, allocation or free.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/nngp.h"
#include "nngp_internal.h"
#include "bf_pairb.h"

namespace {
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(NNGP_EHIP, "%s: %s", what, hipGetErrorString(e));
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// NNGP_ALGO_AUTO: fastest kernel per m, measured on MI355X at N = 1e6 in Z-order (tools/algo_table.py):
// the 2x2-blocked two-lane kernel (bf_pairb.h; left-looking from m = 18, at one wave with 7 factor
// rows in LDS from m = 23) for 1 <= m <= 30 and m = 32 (profiles/r02ap, r03e; m = 25..32 since round 5,
// profiles/r05z3: 0.72 / 1.05 / 2.05 ms per 1e6 rows at m = 25 / 28 / 32 against the four-lane kernel's
// 1.07 / 1.42 / 2.77), four lanes per location at m = 31 (1.68 vs 1.83 ms), one wavefront per location
// above; every kind and dimension.  The general-smoothness Matern kind keeps the four-lane kernel for
// m = 25..32 (its pair-kernel form is right-looking: the table path is not instantiated above 24).
int resolve_algo(int32_t algo, int32_t m, int32_t kind, int32_t dim) {
    (void)dim;
    if (algo != NNGP_ALGO_AUTO) return algo;
    // general-smoothness Matern: the launch's table on the pair kernel for m <= 24 and on the four-lane
    // kernel for 25..32 (since round 5 every nu in (0, 50]: below 2^-64 in t the small-t expansion,
    // nngp_math.h), the wavefront kernel (the direct Bessel evaluation) above.  (A deferred sweep's finalize
    // takes the resolved algo; bf_finalize_pairb refuses a header that is not a pair-kernel sweep of that
    // many rows.)
    if (kind == NNGP_COV_MATERN)
        return m >= 1 && m <= 24 ? nngp::kAlgoPairB : (m >= 25 && m <= 32 ? nngp::kAlgoQuad : nngp::kAlgoWave);
    if (m >= 1 && m <= 32) return m == 31 ? nngp::kAlgoQuad : nngp::kAlgoPairB;
    return nngp::kAlgoWave;
}

// ... for a given smoothness: the Matern table must fit NNGP_MT_MAX_OCT octaves (every nu in (0, 50] since
// the small-t expansion took over below 2^-64; kept as the guard), else the wavefront kernel
int resolve_algo_nu(int32_t algo, int32_t m, int32_t kind, int32_t dim, double nu) {
    const int a = resolve_algo(algo, m, kind, dim);
    if (algo != NNGP_ALGO_AUTO || kind != NNGP_COV_MATERN || (a != nngp::kAlgoPairB && a != nngp::kAlgoQuad)) return a;
    int e0, noct;
    return nu > 0.0 && nu <= NNGP_MATERN_NU_MAX && nngp::matern_table_extent(nu, &e0, &noct) ? a : nngp::kAlgoWave;
}

int64_t bf_blocks(int64_t n_rows, int algo, int m) { return nngp::bf_record_count(n_rows, algo, m); }
}  // namespace

extern "C" {

const char* nngp_version(void) { return "pynngp_amd 0.4.0 gfx950"; }

int32_t nngp_abi_version(void) { return NNGP_ABI_VERSION; }

const char* nngp_last_error(void) { return g_err; }

int32_t nngp_resolve_algo(int32_t algo, int32_t m, int32_t kind, int32_t dim) { return resolve_algo(algo, m, kind, dim); }

int32_t nngp_resolve_algo_nu(int32_t algo, int32_t m, int32_t kind, int32_t dim, double nu) {
    return resolve_algo_nu(algo, m, kind, dim, nu);
}

int nngp_check_partials(const double* p, int64_t* first_bad_row, int64_t* first_bad_index) {
    if (p == nullptr) return fail(NNGP_EINVAL, "partials must be non-null");
    if (first_bad_row != nullptr) *first_bad_row = p[2] >= 0.0 ? (int64_t)p[2] : -1;
    if (first_bad_index != nullptr) *first_bad_index = p[3] >= 0.0 ? (int64_t)p[3] : -1;
    if (p[3] >= 0.0) return fail(NNGP_EINVAL, "neighbour index out of range at location %lld", (long long)p[3]);
    if (p[2] >= 0.0) return fail(NNGP_ENOTPD, "C_N or F not positive definite at location %lld", (long long)p[2]);
    return NNGP_OK;
}

double nngp_loglik_from_partials(const double* p, int64_t n_rows) {
    return -0.5 * ((double)n_rows * 1.8378770664093453 + p[0] + p[1]);
}

size_t nngp_bf_sweep_workspace_bytes(int64_t n_rows, int32_t m, int32_t kind, int32_t dim, int32_t algo) {
    if (n_rows < 0 || m < 0 || m > NNGP_MAX_M) return 0;
    const int a = resolve_algo(algo, m, kind, dim);
    const int64_t nbw = n_rows > 0 ? bf_blocks(n_rows, nngp::kAlgoWave, m) : 0;
    if (kind == NNGP_COV_MATERN && a == nngp::kAlgoPairB) {
        // tile records + exponent sums + the Matern table (AUTO also covers the wavefront kernel's records)
        const size_t pb = nngp::bf_pairb_workspace_bytes(n_rows) + align256(NNGP_MT_BYTES(NNGP_MT_MAX_OCT));
        const size_t wb = align256((size_t)nbw * 4 * sizeof(double));
        return algo == NNGP_ALGO_AUTO && wb > pb ? wb : pb;
    }
    if (kind == NNGP_COV_MATERN && a == nngp::kAlgoQuad) {  // block records + the Matern table
        const int64_t nq = n_rows > 0 ? bf_blocks(n_rows, nngp::kAlgoQuad, m) : 0;
        const size_t qb = align256((size_t)nq * 4 * sizeof(double)) + align256(NNGP_MT_BYTES(NNGP_MT_MAX_OCT));
        const size_t wb = align256((size_t)nbw * 4 * sizeof(double));
        return algo == NNGP_ALGO_AUTO && wb > qb ? wb : qb;
    }
    if (a == nngp::kAlgoPairB) return nngp::bf_pairb_workspace_bytes(n_rows);  // tile records + exponent sums
    const int64_t nb = n_rows > 0 ? bf_blocks(n_rows, a, m) : 0;
    return align256((size_t)nb * 4 * sizeof(double));
}

static int bf_common(const double* coords, int64_t n_points, int32_t dim, const double* qcoords, int64_t n_locs,
                     const int32_t* nbr, const int32_t* order, int64_t n_rows, int32_t m, int64_t i0, int32_t kind,
                     double sigma2, double phi, double tau2, double nu, const double* values, const double* qvalues, double* B,
                     double* F, double* R, double* partials, void* workspace, size_t workspace_bytes, int32_t algo,
                     void* stream) {
    if (coords == nullptr || qcoords == nullptr || workspace == nullptr)
        return fail(NNGP_EINVAL, "coordinates and workspace must be non-null");
    if (dim < 1 || dim > NNGP_MAX_DIM) return fail(NNGP_EUNSUP, "dim=%d outside [1, %d]", dim, NNGP_MAX_DIM);
    if (m < 0 || m > NNGP_MAX_M) return fail(NNGP_EUNSUP, "m=%d outside [0, %d]", m, NNGP_MAX_M);
    if (m > 0 && n_rows > 0 && nbr == nullptr) return fail(NNGP_EINVAL, "nbr must be non-null for m > 0");
    if (n_points < 1 || n_rows < 0 || i0 < 0 || i0 + n_rows > n_locs)
        return fail(NNGP_EINVAL, "rows [%lld, %lld) outside [0, %lld)", (long long)i0, (long long)(i0 + n_rows),
                    (long long)n_locs);
    if (kind < NNGP_COV_EXPONENTIAL || kind > NNGP_COV_MATERN) return fail(NNGP_EINVAL, "unknown kind %d", kind);
    if (!(sigma2 > 0.0) || !(phi > 0.0) || !(tau2 >= 0.0) || !isfinite(sigma2) || !isfinite(phi) || !isfinite(tau2))
        return fail(NNGP_EINVAL, "theta must satisfy sigma2 > 0, phi > 0, tau2 >= 0 (finite)");
    if (kind == NNGP_COV_MATERN && !(nu > 0.0 && nu <= NNGP_MATERN_NU_MAX))
        return fail(NNGP_EINVAL, "the matern kind needs 0 < nu <= %g (nu=%g)", NNGP_MATERN_NU_MAX, nu);
    if (B != nullptr && F == nullptr) return fail(NNGP_EINVAL, "B given without F");
    if (F != nullptr && B == nullptr && m > 0 && n_rows > 0) return fail(NNGP_EINVAL, "F given without B");
    if (R != nullptr && values == nullptr) return fail(NNGP_EINVAL, "R (residuals) needs values");
    if (((uintptr_t)workspace & 255) != 0) return fail(NNGP_EINVAL, "workspace must be 256-byte aligned");
    int a = resolve_algo_nu(algo, m, kind, dim, nu);
    if (a != nngp::kAlgoLane && a != nngp::kAlgoWave && a != nngp::kAlgoQuad && a != nngp::kAlgoPairB)
        return fail(NNGP_EINVAL, "unknown algo %d", algo);
    if (kind == NNGP_COV_MATERN && a != nngp::kAlgoWave && a != nngp::kAlgoPairB && a != nngp::kAlgoQuad)
        return fail(NNGP_EUNSUP, "the matern kind runs on the pair (m <= 24), four-lane (25..32) or wavefront kernel, "
                                 "not algo %d", algo);
    if (kind == NNGP_COV_MATERN && (a == nngp::kAlgoPairB || a == nngp::kAlgoQuad)) {
        int e0, noct;
        if (!nngp::matern_table_extent(nu, &e0, &noct))
            return fail(NNGP_EUNSUP, "matern nu=%g needs %d table octaves (> %d; nu below ~%g): use NNGP_ALGO_AUTO or "
                                     "WAVE", nu, noct, NNGP_MT_MAX_OCT, NNGP_MT_NU_MIN);
    }
    const bool classic = dim == 2 && kind <= NNGP_COV_MATERN32;
    if (a == nngp::kAlgoLane && !classic)
        return fail(NNGP_EUNSUP, "the lane kernel serves 2-D exponential and Matern-3/2 only "
                                 "(kind=%d, dim=%d): use NNGP_ALGO_AUTO, PAIRB, QUAD or WAVE", kind, dim);
    if (a == nngp::kAlgoLane && (m < 1 || m > nngp::kLaneMaxM))
        return fail(NNGP_EUNSUP, "lane kernel needs 1 <= m <= %d (m=%d)", nngp::kLaneMaxM, m);
    if (a == nngp::kAlgoQuad && !nngp::bf_group_supported(m, 4))
        return fail(NNGP_EUNSUP, "no 4-lane kernel instantiated for m=%d (25..32)", m);
    if (a == nngp::kAlgoPairB && !nngp::bf_pairb_supported(m))
        return fail(NNGP_EUNSUP, "no blocked pair kernel instantiated for m=%d", m);
    if (a == nngp::kAlgoPairB && kind == NNGP_COV_MATERN && m > 24)
        return fail(NNGP_EUNSUP, "the matern kind runs on the pair kernel for m <= 24 (m=%d): use NNGP_ALGO_AUTO or "
                                 "QUAD", m);
    const size_t need = nngp_bf_sweep_workspace_bytes(n_rows, m, kind, dim, algo);
    if (workspace_bytes < need)
        return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes, need);

    hipStream_t s = (hipStream_t)stream;
    nngp::BfArgs args{coords, n_points, nbr, n_rows, i0, m, kind, dim, sigma2, phi, tau2, nu, order, values, qcoords,
                      qvalues, B, F, R, partials, (double*)workspace};
    hipError_t e = nngp::bf_launch(args, a, s);
    if (e != hipSuccess) return hip_fail(e, "bf_sweep launch");
    return NNGP_OK;
}

int nngp_bf_sweep(const double* coords, int64_t n_points, int32_t dim, const int32_t* nbr, const int32_t* order,
                  int64_t n_rows, int32_t m, int64_t i0, int32_t kind, double sigma2, double phi, double tau2,
                  double nu, const double* values, double* B, double* F, double* R, double* partials, void* workspace,
                  size_t workspace_bytes, int32_t algo, void* stream) {
    return bf_common(coords, n_points, dim, coords, n_points, nbr, order, n_rows, m, i0, kind, sigma2, phi, tau2, nu,
                     values, values, B, F, R, partials, workspace, workspace_bytes, algo, stream);
}

int nngp_bf_cross(const double* ref, int64_t n_ref, int32_t dim, const double* query, int64_t n_query,
                  const int32_t* nbr, const int32_t* order, int64_t n_rows, int32_t m, int64_t q0, int32_t kind,
                  double sigma2, double phi, double tau2, double nu, const double* ref_values,
                  const double* query_values, double* B, double* F, double* R, double* partials, void* workspace,
                  size_t workspace_bytes, int32_t algo, void* stream) {
    if (query_values != nullptr && ref_values == nullptr)
        return fail(NNGP_EINVAL, "query_values need ref_values");
    return bf_common(ref, n_ref, dim, query, n_query, nbr, order, n_rows, m, q0, kind, sigma2, phi, tau2, nu, ref_values,
                     query_values, B, F, R, partials, workspace, workspace_bytes, algo, stream);
}

int nngp_pair_plan_supported(int32_t m, int32_t kind, int32_t dim) {
    return nngp::bf_pairb_planned_supported(m, kind, dim) ? 1 : 0;
}

size_t nngp_pair_plan_bytes(int64_t n_rows, int32_t m, int32_t dim) {
    if (n_rows < 0 || n_rows > INT32_MAX || !nngp::bf_pairb_planned_supported(m, 0, dim)) return 0;
    return (size_t)nngp::plan_total_bytes(n_rows, m);
}

int nngp_pair_plan_build(const int32_t* nbr, const int32_t* order, int64_t n_rows, int32_t m, int64_t i0,
                         int64_t n_points, int32_t dim, void* plan, size_t plan_bytes, int64_t* info, void* stream) {
    if (plan == nullptr || info == nullptr || (n_rows > 0 && nbr == nullptr))
        return fail(NNGP_EINVAL, "plan, info (and nbr for n_rows > 0) must be non-null");
    if (!nngp::bf_pairb_planned_supported(m, 0, dim))
        return fail(NNGP_EUNSUP, "pair plans serve 2 <= m <= 17, dim 1..3 (m=%d, dim=%d)", m, dim);
    if (n_rows < 0 || n_rows > INT32_MAX || i0 < 0 || n_points < 1 || i0 + n_rows > n_points || n_points > INT32_MAX)
        return fail(NNGP_EINVAL, "rows [%lld, %lld) outside [0, %lld) (or n_rows / n_points >= 2^31)", (long long)i0,
                    (long long)(i0 + n_rows), (long long)n_points);
    if (((uintptr_t)plan & 255) != 0) return fail(NNGP_EINVAL, "plan must be 256-byte aligned");
    const size_t need = (size_t)nngp::plan_total_bytes(n_rows, m);
    if (plan_bytes < need) return fail(NNGP_EINVAL, "plan too small: %zu < %zu bytes", plan_bytes, need);
    hipStream_t s = (hipStream_t)stream;
    const nngp::PairbTiling tl = nngp::pairb_tiling(n_rows, m, 0);
    if (tl.tiles != nngp::plan_regions(n_rows)) return fail(NNGP_EUNSUP, "plan regions differ from the pair tiling");
    hipError_t e = nngp::pair_plan_build_launch(nbr, order, n_rows, m, dim, i0, n_points, tl.q, tl.rem, plan, s);
    if (e != hipSuccess) return hip_fail(e, "pair_plan build");
    nngp::PlanHeader h;
    e = hipMemcpyAsync(&h, plan, sizeof h, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "pair_plan counts");
    info[0] = h.n_planned;
    info[1] = h.n_direct;
    info[2] = n_rows;
    info[3] = m;
    info[4] = dim;
    info[5] = i0;
    info[6] = n_points;
    info[7] = nngp::kPlanMagic;
    info[8] = (int64_t)(uintptr_t)nbr;
    info[9] = (int64_t)(uintptr_t)order;
    return NNGP_OK;
}

int nngp_bf_sweep_plan(const double* coords, int64_t n_points, int32_t dim, const int32_t* nbr, const int32_t* order,
                       int64_t n_rows, int32_t m, int64_t i0, int32_t kind, double sigma2, double phi, double tau2,
                       const double* values, double* B, double* F, double* R, double* partials, void* workspace,
                       size_t workspace_bytes, const void* plan, size_t plan_bytes, const int64_t* info,
                       void* stream) {
    if (coords == nullptr || workspace == nullptr || plan == nullptr || info == nullptr)
        return fail(NNGP_EINVAL, "coordinates, workspace, plan and info must be non-null");
    if (info[7] != nngp::kPlanMagic || info[2] != n_rows || info[3] != m || info[4] != dim || info[5] != i0 ||
        info[6] != n_points)
        return fail(NNGP_EINVAL, "the plan was built for (n_rows %lld, m %lld, dim %lld, i0 %lld, n_points %lld), not "
                                 "this sweep's (%lld, %d, %d, %lld, %lld)", (long long)info[2], (long long)info[3],
                    (long long)info[4], (long long)info[5], (long long)info[6], (long long)n_rows, m, dim,
                    (long long)i0, (long long)n_points);
    if (info[8] != (int64_t)(uintptr_t)nbr || info[9] != (int64_t)(uintptr_t)order)
        return fail(NNGP_EINVAL, "stale plan: it was built for other nbr / order buffers (rebuild it with the "
                                 "sweep's neighbour sets)");
    if (!nngp::bf_pairb_planned_supported(m, kind, dim))
        return fail(NNGP_EUNSUP, "planned sweeps serve kinds 0..4, 2 <= m <= 17, dim 1..3 (kind=%d)", kind);
    if (plan_bytes < (size_t)nngp::plan_total_bytes(n_rows, m)) return fail(NNGP_EINVAL, "plan too small");
    const int64_t nreg = nngp::plan_regions(n_rows);
    if (info[0] < 0 || info[1] < 0 || info[0] + info[1] != nreg)
        return fail(NNGP_EINVAL, "plan counts %lld + %lld != %lld tiles", (long long)info[0], (long long)info[1],
                    (long long)nreg);
    // the unplanned sweep's argument checks (same kernel family, same workspace)
    if (m < 1 || (n_rows > 0 && nbr == nullptr)) return fail(NNGP_EINVAL, "nbr must be non-null");
    if (!(sigma2 > 0.0) || !(phi > 0.0) || !(tau2 >= 0.0) || !isfinite(sigma2) || !isfinite(phi) || !isfinite(tau2))
        return fail(NNGP_EINVAL, "theta must satisfy sigma2 > 0, phi > 0, tau2 >= 0 (finite)");
    if (B != nullptr && F == nullptr) return fail(NNGP_EINVAL, "B given without F");
    if (F != nullptr && B == nullptr && n_rows > 0) return fail(NNGP_EINVAL, "F given without B");
    if (R != nullptr && values == nullptr) return fail(NNGP_EINVAL, "R (residuals) needs values");
    if (((uintptr_t)workspace & 255) != 0) return fail(NNGP_EINVAL, "workspace must be 256-byte aligned");
    const size_t need = nngp_bf_sweep_workspace_bytes(n_rows, m, kind, dim, NNGP_ALGO_PAIRB);
    if (workspace_bytes < need) return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes, need);
    const uint8_t* p = (const uint8_t*)plan;
    const int64_t sb = nngp::plan_slot_bytes(m);
    const int32_t* planned = (const int32_t*)(p + nngp::kPlanGlobalHdr + nreg * sb);
    nngp::PlanLaunch pl{p, nreg, info[0], info[1], sb, planned, planned + nreg};
    nngp::BfArgs args{coords, n_points, nbr, n_rows, i0, m, kind, dim, sigma2, phi, tau2, 0.0, order, values, coords,
                      values, B, F, R, partials, (double*)workspace};
    hipError_t e = nngp::bf_launch_planned(args, pl, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "bf_sweep_plan launch");
    return NNGP_OK;
}

int64_t nngp_joint_entries(int32_t m) { return m < 0 ? 0 : (int64_t)(m + 1) * (m + 2) / 2; }

int nngp_joint_dist(const double* coords, int64_t n_points, int32_t dim, const double* qcoords, int64_t n_locs,
                    const int32_t* nbr, const int32_t* order, int64_t n_rows, int32_t m, int64_t i0, double* dist,
                    void* stream) {
    if (coords == nullptr || qcoords == nullptr || dist == nullptr || (m > 0 && n_rows > 0 && nbr == nullptr))
        return fail(NNGP_EINVAL, "coords, qcoords, dist (and nbr for m > 0) must be non-null");
    if (dim < 1 || dim > NNGP_MAX_DIM) return fail(NNGP_EUNSUP, "dim=%d outside [1, %d]", dim, NNGP_MAX_DIM);
    if (m < 0 || m > NNGP_MAX_M) return fail(NNGP_EUNSUP, "m=%d outside [0, %d]", m, NNGP_MAX_M);
    if (n_points < 1 || n_rows < 0 || i0 < 0 || i0 + n_rows > n_locs)
        return fail(NNGP_EINVAL, "rows [%lld, %lld) outside [0, %lld)", (long long)i0, (long long)(i0 + n_rows),
                    (long long)n_locs);
    hipError_t e = nngp::joint_dist_launch(coords, n_points, dim, qcoords, nbr, order, n_rows, m, i0, dist,
                                           (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "joint_dist launch");
    return NNGP_OK;
}

int nngp_matern_eval(const double* u, int64_t n, double nu, double* out, void* stream) {
    if (n < 0 || (n > 0 && (u == nullptr || out == nullptr))) return fail(NNGP_EINVAL, "bad n or null pointer");
    if (!(nu > 0.0 && nu <= NNGP_MATERN_NU_MAX))
        return fail(NNGP_EINVAL, "the matern correlation needs 0 < nu <= %g (nu=%g)", NNGP_MATERN_NU_MAX, nu);
    hipError_t e = nngp::matern_eval_launch(u, n, nu, out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "matern_eval launch");
    return NNGP_OK;
}

size_t nngp_bf_sweep_blocks_workspace_bytes(int64_t n_rows) {
    // enough for either kernel: bf_pairb's tile records (m <= 24) or the four-lane kernel's block
    // records (m = 25..32)
    if (n_rows < 0) return 0;
    const size_t pb = nngp::bf_pairb_workspace_bytes(n_rows);
    const size_t gb = align256((size_t)nngp::bf_group_blocks(n_rows, 4) * 4 * sizeof(double));
    return pb > gb ? pb : gb;
}

int nngp_bf_sweep_blocks(const double* cov, const int32_t* nbr, const int32_t* order, int64_t n_points, int64_t n_rows,
                         int32_t m, int64_t i0, int64_t n_locs, const double* values, const double* qvalues, double* B,
                         double* F, double* R, double* partials, void* workspace, size_t workspace_bytes,
                         void* stream) {
    if (cov == nullptr || workspace == nullptr || partials == nullptr || (n_rows > 0 && nbr == nullptr))
        return fail(NNGP_EINVAL, "cov, nbr, partials and workspace must be non-null");
    const bool group = nngp::bf_group_blocks_supported(m);
    if (!nngp::bf_pairb_blocks_supported(m) && !group)
        return fail(NNGP_EUNSUP, "covariance-block sweeps need 1 <= m <= 32 (m=%d)", m);
    if (n_points < 1 || n_rows < 0 || i0 < 0 || i0 + n_rows > n_locs)
        return fail(NNGP_EINVAL, "rows [%lld, %lld) outside [0, %lld)", (long long)i0, (long long)(i0 + n_rows),
                    (long long)n_locs);
    if (B != nullptr && F == nullptr) return fail(NNGP_EINVAL, "B given without F");
    if (F != nullptr && B == nullptr) return fail(NNGP_EINVAL, "F given without B");
    if (R != nullptr && values == nullptr) return fail(NNGP_EINVAL, "R (residuals) needs values");
    if (((uintptr_t)workspace & 255) != 0) return fail(NNGP_EINVAL, "workspace must be 256-byte aligned");
    if (workspace_bytes < nngp_bf_sweep_blocks_workspace_bytes(n_rows))
        return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes,
                    nngp_bf_sweep_blocks_workspace_bytes(n_rows));
    hipStream_t s = (hipStream_t)stream;
    if (n_rows == 0) {
        hipError_t e = nngp::bf_finalize_launch((const double*)workspace, 0, partials, s);
        return e == hipSuccess ? NNGP_OK : hip_fail(e, "bf_finalize launch");
    }
    nngp::BfArgs args{nullptr, n_points, nbr, n_rows, i0, m, NNGP_KIND_BLOCKS, 2, 1.0, 1.0, 0.0, 0.0, order, values,
                      nullptr, qvalues, B, F, R, partials, (double*)workspace, cov};
    if (!(group ? nngp::bf_group_blocks_launch(args, s) : nngp::bf_pairb_blocks_launch(args, s)))
        return fail(NNGP_EUNSUP, "no covariance-block kernel for m=%d", m);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = group ? nngp::bf_finalize_launch((const double*)workspace, nngp::bf_group_blocks(n_rows, 4), partials, s)
                  : nngp::bf_finalize_pairb_launch(workspace, n_rows, partials, s);
    if (e != hipSuccess) return hip_fail(e, "bf_sweep_blocks launch");
    return NNGP_OK;
}

int nngp_bf_finalize(const void* workspace, size_t workspace_bytes, int64_t n_rows, int32_t m, int32_t kind,
                     int32_t dim, int32_t algo, double* partials, void* stream) {
    if (workspace == nullptr || partials == nullptr) return fail(NNGP_EINVAL, "workspace and partials must be non-null");
    if (n_rows < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n_rows or m");
    if (dim < 1 || dim > NNGP_MAX_DIM || kind < NNGP_COV_EXPONENTIAL || kind > NNGP_COV_MATERN)
        return fail(NNGP_EINVAL, "bad kind %d or dim %d", kind, dim);
    if (kind == NNGP_COV_MATERN && algo == NNGP_ALGO_AUTO)
        return fail(NNGP_EINVAL, "the matern kind's kernel depends on nu: pass the sweep's resolved algo "
                                 "(nngp_resolve_algo_nu), not NNGP_ALGO_AUTO");
    const int a = resolve_algo(algo, m, kind, dim);
    if (a != nngp::kAlgoLane && a != nngp::kAlgoWave && a != nngp::kAlgoQuad && a != nngp::kAlgoPairB)
        return fail(NNGP_EINVAL, "unknown algo %d", algo);
    const size_t need = nngp_bf_sweep_workspace_bytes(n_rows, m, kind, dim, algo);
    if (workspace_bytes < need)
        return fail(NNGP_EINVAL, "workspace of %zu bytes is smaller than the %zu the sweep (n_rows=%lld, m=%d, "
                                 "kind=%d, dim=%d, algo=%d) needs", workspace_bytes, need, (long long)n_rows, m, kind,
                    dim, algo);
    hipError_t e = a == nngp::kAlgoPairB && n_rows > 0
                       ? nngp::bf_finalize_pairb_launch((void*)workspace, n_rows, partials, (hipStream_t)stream)
                       : nngp::bf_finalize_launch((const double*)workspace, nngp::bf_record_count(n_rows, a, m),
                                                  partials, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "bf_finalize launch");
    return NNGP_OK;
}

int nngp_combine_partials_batch(const double* gathered, int32_t world, int64_t n_slots, double* partials,
                                void* stream) {
    if (gathered == nullptr || partials == nullptr) return fail(NNGP_EINVAL, "gathered and partials must be non-null");
    if (world < 1) return fail(NNGP_EINVAL, "world=%d < 1", world);
    if (n_slots < 0) return fail(NNGP_EINVAL, "n_slots=%lld < 0", (long long)n_slots);
    hipError_t e = nngp::combine_partials_launch(gathered, world, n_slots, partials, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "combine_partials launch");
    return NNGP_OK;
}

int nngp_combine_partials(const double* gathered, int32_t world, double* partials, void* stream) {
    return nngp_combine_partials_batch(gathered, world, 1, partials, stream);
}

size_t nngp_reverse_workspace_bytes(int64_t n, int32_t m) {
    if (n < 0 || m < 0 || n * (int64_t)m > INT32_MAX) return 0;
    return nngp::reverse_workspace_bytes(n, m);
}

int nngp_reverse_neighbors(const int32_t* nbr, int64_t n, int32_t m, int32_t* off, int32_t* rev_j, int32_t* rev_k,
                           void* workspace, size_t workspace_bytes, void* stream) {
    if (off == nullptr || workspace == nullptr) return fail(NNGP_EINVAL, "off and workspace must be non-null");
    if (n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n=%lld or m=%d", (long long)n, m);
    if (n * (int64_t)m > INT32_MAX) return fail(NNGP_EUNSUP, "n*m must be < 2^31");
    if (n * m > 0 && (nbr == nullptr || rev_j == nullptr || rev_k == nullptr))
        return fail(NNGP_EINVAL, "nbr, rev_j and rev_k must be non-null");
    if (((uintptr_t)workspace & 255) != 0) return fail(NNGP_EINVAL, "workspace must be 256-byte aligned");
    const size_t need = nngp::reverse_workspace_bytes(n, m);
    if (need == 0 || workspace_bytes < need)
        return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes, need);
    hipError_t e = nngp::reverse_launch(nbr, n, m, off, rev_j, rev_k, workspace, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "reverse_neighbors launch");
    return NNGP_OK;
}

int64_t nngp_color_moral_graph(const int32_t* nbr, const int32_t* off, const int32_t* rev_j, int64_t n, int32_t m,
                               int32_t* color) {
    if (n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n or m");
    if (n > 0 && (off == nullptr || color == nullptr || (m > 0 && (nbr == nullptr || rev_j == nullptr))))
        return fail(NNGP_EINVAL, "null host pointer");
    return nngp::color_moral_graph_host(nbr, off, rev_j, n, m, color);
}

int64_t nngp_color_moral_graph_dev(const int32_t* nbr, const int32_t* off, const int32_t* rev_j, int64_t n, int32_t m,
                                   int32_t* color, void* workspace, size_t workspace_bytes, void* stream) {
    if (n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n or m");
    if (n > 0 && (off == nullptr || color == nullptr || workspace == nullptr || (m > 0 && (nbr == nullptr || rev_j == nullptr))))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (workspace_bytes < 256) return fail(NNGP_EINVAL, "workspace too small: %zu < 256 bytes", workspace_bytes);
    hipError_t e;
    const int64_t nc = nngp::color_moral_graph_device(nbr, off, rev_j, n, m, color, workspace, (hipStream_t)stream, &e);
    if (nc == -2) return hip_fail(e, "color_moral_graph rounds");
    if (nc == -1) return fail(NNGP_EUNSUP, "more than 256 colours: colour on the host (nngp_color_moral_graph)");
    return nc;
}

size_t nngp_gibbs_prep_bytes(int64_t n, int32_t m) {
    if (n < 0 || m < 0 || m > NNGP_MAX_M) return 0;
    return nngp::gibbs_prep_bytes(n, m);
}

int nngp_gibbs_prepare(const double* B, const double* Ft, const int32_t* off, const int32_t* rev_j,
                       const int32_t* rev_k, const int32_t* order, int64_t n, int32_t m, void* prep,
                       size_t prep_bytes, void* stream) {
    if (Ft == nullptr || off == nullptr || prep == nullptr || (m > 0 && (B == nullptr || rev_j == nullptr ||
                                                                          rev_k == nullptr)))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n or m");
    if (((uintptr_t)prep & 255) != 0) return fail(NNGP_EINVAL, "prep must be 256-byte aligned");
    if (prep_bytes < nngp::gibbs_prep_bytes(n, m))
        return fail(NNGP_EINVAL, "prep too small: %zu < %zu bytes", prep_bytes, nngp::gibbs_prep_bytes(n, m));
    hipError_t e = nngp::gibbs_prepare_launch(B, Ft, off, rev_j, rev_k, order, n, m, prep, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_prepare launch");
    return NNGP_OK;
}

int nngp_gibbs_prepare_range(const double* B, const double* Ft, const int32_t* off, const int32_t* rev_j,
                             const int32_t* rev_k, int64_t n, int32_t m, int64_t row0, int64_t row1, void* prep,
                             size_t prep_bytes, void* stream) {
    if (Ft == nullptr || off == nullptr || prep == nullptr || (m > 0 && (B == nullptr || rev_j == nullptr ||
                                                                          rev_k == nullptr)))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n or m");
    if (row0 < 0 || row1 < row0 || row1 > n) return fail(NNGP_EINVAL, "rows [%lld, %lld) outside [0, %lld)",
                                                         (long long)row0, (long long)row1, (long long)n);
    if (((uintptr_t)prep & 255) != 0) return fail(NNGP_EINVAL, "prep must be 256-byte aligned");
    if (prep_bytes < nngp::gibbs_prep_bytes(n, m))
        return fail(NNGP_EINVAL, "prep too small: %zu < %zu bytes", prep_bytes, nngp::gibbs_prep_bytes(n, m));
    hipError_t e = nngp::gibbs_prepare_range_launch(B, Ft, off, rev_j, rev_k, n, m, row0, row1, prep,
                                                    (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_prepare_range launch");
    return NNGP_OK;
}

static int gibbs_w_color_common(const int32_t* member_rows, int64_t n_members, const void* prep, int64_t n,
                                int32_t m, double sigma2, double tau2, const double* var, const double* yres,
                                const double* noise_w, double* w, double* r, const int32_t* rev_j, const double* z,
                                uint64_t seed, uint64_t sweep, double* w_out, void* stream) {
    if (n_members < 0 || n < 0 || m < 0 || m > NNGP_MAX_M || n_members > n)
        return fail(NNGP_EINVAL, "bad n_members, n or m");
    if (n_members == 0) return NNGP_OK;
    if (member_rows == nullptr || prep == nullptr || yres == nullptr || w == nullptr || r == nullptr ||
        (m > 0 && rev_j == nullptr))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (((uintptr_t)member_rows & 15) != 0) return fail(NNGP_EINVAL, "member_rows must be 16-byte aligned");
    if (var == nullptr && (!(sigma2 > 0.0) || !(tau2 > 0.0) || !isfinite(sigma2) || !isfinite(tau2)))
        return fail(NNGP_EINVAL, "need sigma2 > 0 and tau2 > 0 (finite)");
    hipError_t e = nngp::gibbs_w_color_launch(member_rows, n_members, prep, n, m, var ? 1.0 : sigma2,
                                              var ? 1.0 : tau2, yres, noise_w, w, r, rev_j, z, seed, sweep, w_out, var,
                                              (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_w_color launch");
    return NNGP_OK;
}

int nngp_gibbs_w_color(const int32_t* member_rows, int64_t n_members, const void* prep, int64_t n, int32_t m,
                       double sigma2, double tau2, const double* yres, const double* noise_w, double* w, double* r,
                       const int32_t* rev_j, const double* z, uint64_t seed, uint64_t sweep, double* w_out,
                       void* stream) {
    return gibbs_w_color_common(member_rows, n_members, prep, n, m, sigma2, tau2, nullptr, yres, noise_w, w, r, rev_j,
                                z, seed, sweep, w_out, stream);
}

int nngp_gibbs_w_color_dev(const int32_t* member_rows, int64_t n_members, const void* prep, int64_t n, int32_t m,
                           const double* var, const double* yres, const double* noise_w, double* w, double* r,
                           const int32_t* rev_j, const double* z, double* w_out, void* stream) {
    if (var == nullptr || (n_members > 0 && z == nullptr)) return fail(NNGP_EINVAL, "var and z must be given");
    return gibbs_w_color_common(member_rows, n_members, prep, n, m, 1.0, 1.0, var, yres, noise_w, w, r, rev_j, z, 0, 0,
                                w_out, stream);
}

int nngp_gibbs_w_apply(const int32_t* rows, int64_t n_rows, const double* w_src, const double* B, int64_t n, int32_t m,
                       double* w, double* r, const int32_t* rev_j, const int32_t* rev_k, void* stream) {
    if (n_rows < 0 || n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n_rows, n or m");
    if (n_rows == 0) return NNGP_OK;
    if (rows == nullptr || w_src == nullptr || w == nullptr || r == nullptr ||
        (m > 0 && (B == nullptr || rev_j == nullptr || rev_k == nullptr)))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (((uintptr_t)rows & 15) != 0) return fail(NNGP_EINVAL, "rows must be 16-byte aligned");
    hipError_t e = nngp::gibbs_w_apply_launch(rows, n_rows, w_src, B, m, w, r, rev_j, rev_k, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_w_apply launch");
    return NNGP_OK;
}

int nngp_gibbs_member_rows(const int32_t* members, int64_t n, const int32_t* off, int32_t* member_rows, void* stream) {
    if (n < 0 || (n > 0 && (members == nullptr || off == nullptr || member_rows == nullptr)))
        return fail(NNGP_EINVAL, "bad n or null pointer argument");
    if (((uintptr_t)member_rows & 15) != 0) return fail(NNGP_EINVAL, "member_rows must be 16-byte aligned");
    hipError_t e = nngp::gibbs_member_rows_launch(members, n, off, member_rows, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_member_rows launch");
    return NNGP_OK;
}

int nngp_gibbs_w_sweep(const int32_t* member_rows, const int32_t* color_off_host, int32_t n_colors, const void* prep,
                       int64_t n, int32_t m, double sigma2, double tau2, const double* yres, const double* noise_w,
                       double* w, double* r, const int32_t* rev_j, const double* z, uint64_t seed, uint64_t sweep,
                       void* stream) {
    if (member_rows == nullptr || color_off_host == nullptr || prep == nullptr || yres == nullptr || w == nullptr ||
        r == nullptr || (m > 0 && rev_j == nullptr))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (((uintptr_t)member_rows & 15) != 0) return fail(NNGP_EINVAL, "member_rows must be 16-byte aligned");
    if (n_colors < 0 || n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n_colors, n or m");
    if (n_colors > 0 && color_off_host[n_colors] > n) return fail(NNGP_EINVAL, "colour offsets exceed n");
    for (int c = 0; c <= n_colors; ++c)
        if (color_off_host[c] < 0) return fail(NNGP_EINVAL, "negative colour offset");
    if (!(sigma2 > 0.0) || !(tau2 > 0.0) || !isfinite(sigma2) || !isfinite(tau2))
        return fail(NNGP_EINVAL, "need sigma2 > 0 and tau2 > 0 (finite)");
    hipError_t e = nngp::gibbs_w_sweep_launch(member_rows, n_colors, color_off_host, prep, n, m, sigma2, tau2, yres,
                                              noise_w, w, r, rev_j, z, seed, sweep, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_w_sweep launch");
    return NNGP_OK;
}

int nngp_gibbs_w_sweep_tiles(const int32_t* tiles, const int32_t* phase_off_host, const int32_t* phase_lds_host,
                             int32_t n_phases, const int32_t* tinfo, const int32_t* tstep, int32_t ecap,
                             const int32_t* tfp, const int32_t* off, const int32_t* rev_loc, const void* prep,
                             int64_t n, int32_t m, int64_t n_entries, double sigma2, double tau2, const double* yres,
                             const double* noise_w, double* w, double* r, const double* z, void* stream) {
    if (tiles == nullptr || phase_off_host == nullptr || phase_lds_host == nullptr || tinfo == nullptr ||
        tstep == nullptr || tfp == nullptr || off == nullptr || prep == nullptr || yres == nullptr || w == nullptr ||
        r == nullptr || z == nullptr || (n_entries > 0 && rev_loc == nullptr))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (n_phases < 0 || n < 0 || m < 0 || m > NNGP_MAX_M || n_entries < 0 || n_entries > n * (int64_t)m)
        return fail(NNGP_EINVAL, "bad n_phases, n, m or n_entries");
    if (ecap < 0 || ecap > 2048) return fail(NNGP_EINVAL, "ecap=%d outside [0, 2048] (entries of one step)", ecap);
    if (((uintptr_t)tinfo & 15) != 0) return fail(NNGP_EINVAL, "tinfo must be 16-byte aligned");
    for (int p = 0; p < n_phases; ++p) {
        if (phase_off_host[p + 1] < phase_off_host[p]) return fail(NNGP_EINVAL, "phase offsets must not decrease");
        if (phase_lds_host[p] < 0 || phase_lds_host[p] > 160 * 1024)
            return fail(NNGP_EINVAL, "phase %d needs %d B of LDS (> 160 KB)", p, phase_lds_host[p]);
    }
    if (!(sigma2 > 0.0) || !(tau2 > 0.0) || !isfinite(sigma2) || !isfinite(tau2))
        return fail(NNGP_EINVAL, "need sigma2 > 0 and tau2 > 0 (finite)");
    hipError_t e = nngp::gibbs_tile_sweep_launch(tiles, phase_off_host, phase_lds_host, n_phases, tinfo, tstep, ecap,
                                                 tfp, off, rev_loc, prep, n, m, n_entries, sigma2, tau2, yres, noise_w,
                                                 w, r, z, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_tile_sweep launch");
    return NNGP_OK;
}

int nngp_gibbs_w_sweep_chains(const int32_t* member_rows, const int32_t* color_off_host, int32_t n_colors,
                              int32_t chains, const void* const* prep, int64_t n, int32_t m, const double* sigma2,
                              const double* tau2, const double* const* yres, const double* noise_w, double* const* w,
                              double* const* r, const int32_t* rev_j, const double* const* z, void* stream) {
    if (chains < 1 || chains > 8) return fail(NNGP_EINVAL, "chains=%d outside [1, 8]", chains);
    if (member_rows == nullptr || color_off_host == nullptr || prep == nullptr || sigma2 == nullptr ||
        tau2 == nullptr || yres == nullptr || w == nullptr || r == nullptr || z == nullptr ||
        (m > 0 && rev_j == nullptr))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (((uintptr_t)member_rows & 15) != 0) return fail(NNGP_EINVAL, "member_rows must be 16-byte aligned");
    if (n_colors < 0 || n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n_colors, n or m");
    if (n_colors > 0 && color_off_host[n_colors] > n) return fail(NNGP_EINVAL, "colour offsets exceed n");
    for (int c = 0; c <= n_colors; ++c)
        if (color_off_host[c] < 0) return fail(NNGP_EINVAL, "negative colour offset");
    for (int c = 0; c < chains; ++c) {
        if (prep[c] == nullptr || yres[c] == nullptr || w[c] == nullptr || r[c] == nullptr || z[c] == nullptr)
            return fail(NNGP_EINVAL, "null pointer for chain %d", c);
        if (((uintptr_t)prep[c] & 255) != 0) return fail(NNGP_EINVAL, "prep[%d] must be 256-byte aligned", c);
        if (!(sigma2[c] > 0.0) || !(tau2[c] > 0.0) || !isfinite(sigma2[c]) || !isfinite(tau2[c]))
            return fail(NNGP_EINVAL, "chain %d needs sigma2 > 0 and tau2 > 0 (finite)", c);
    }
    hipError_t e = nngp::gibbs_w_sweep_chains_launch(member_rows, n_colors, color_off_host, chains, prep, n, m, sigma2,
                                                     tau2, yres, noise_w, w, r, rev_j, z, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_w_sweep_chains launch");
    return NNGP_OK;
}

int nngp_gibbs_w_sweep_chains_il(const int32_t* member_rows, const int32_t* color_off_host, int32_t n_colors,
                                 int32_t chains, const void* const* prep, int64_t n, int32_t m, const double* sigma2,
                                 const double* tau2, const double* const* yres, const double* noise_w, double* w_il,
                                 double* r_il, const int32_t* rev_j, const double* const* z, void* stream) {
    if (chains < 1 || chains > 8) return fail(NNGP_EINVAL, "chains=%d outside [1, 8]", chains);
    if (member_rows == nullptr || color_off_host == nullptr || prep == nullptr || sigma2 == nullptr ||
        tau2 == nullptr || yres == nullptr || w_il == nullptr || r_il == nullptr || z == nullptr ||
        (m > 0 && rev_j == nullptr))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (((uintptr_t)member_rows & 15) != 0) return fail(NNGP_EINVAL, "member_rows must be 16-byte aligned");
    if (((uintptr_t)w_il & 15) != 0 || ((uintptr_t)r_il & 15) != 0)  // (read and written as 16-byte pairs)
        return fail(NNGP_EINVAL, "w_il / r_il must be 16-byte aligned");
    if (n_colors < 0 || n < 0 || m < 0 || m > NNGP_MAX_M) return fail(NNGP_EINVAL, "bad n_colors, n or m");
    if (n_colors > 0 && color_off_host[n_colors] > n) return fail(NNGP_EINVAL, "colour offsets exceed n");
    for (int c = 0; c <= n_colors; ++c)
        if (color_off_host[c] < 0) return fail(NNGP_EINVAL, "negative colour offset");
    for (int c = 0; c < chains; ++c) {
        if (prep[c] == nullptr || yres[c] == nullptr || z[c] == nullptr)
            return fail(NNGP_EINVAL, "null pointer for chain %d", c);
        if (((uintptr_t)prep[c] & 255) != 0) return fail(NNGP_EINVAL, "prep[%d] must be 256-byte aligned", c);
        if (!(sigma2[c] > 0.0) || !(tau2[c] > 0.0) || !isfinite(sigma2[c]) || !isfinite(tau2[c]))
            return fail(NNGP_EINVAL, "chain %d needs sigma2 > 0 and tau2 > 0 (finite)", c);
    }
    hipError_t e = nngp::gibbs_w_sweep_chains_launch(member_rows, n_colors, color_off_host, chains, prep, n, m, sigma2,
                                                     tau2, yres, noise_w, nullptr, nullptr, rev_j, z,
                                                     (hipStream_t)stream, w_il, r_il);
    if (e != hipSuccess) return hip_fail(e, "gibbs_w_sweep_chains_il launch");
    return NNGP_OK;
}

int nngp_gibbs_normals(int64_t n, uint64_t seed, uint64_t sweep, double* z, void* stream) {
    if (n < 0 || (n > 0 && z == nullptr)) return fail(NNGP_EINVAL, "bad n or null z");
    hipError_t e = nngp::philox_normals_launch(n, seed, sweep, z, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_normals launch");
    return NNGP_OK;
}

size_t nngp_gibbs_stats_workspace_bytes(int64_t n, int32_t p) {
    if (n < 1 || p < 0 || p > 62) return 0;
    return nngp::gibbs_stats_workspace_bytes(n, p);
}

int nngp_gibbs_stats(int64_t n, const double* r, const double* Ft, const double* yres, const double* y, const double* X,
                     int32_t p, const double* w, const double* noise_w, double* out, void* workspace,
                     size_t workspace_bytes, void* stream) {
    if (r == nullptr || Ft == nullptr || yres == nullptr || w == nullptr || out == nullptr || workspace == nullptr ||
        (p > 0 && (X == nullptr || y == nullptr)))
        return fail(NNGP_EINVAL, "null pointer argument");
    if (n < 1 || p < 0 || p > 62) return fail(NNGP_EINVAL, "bad n or p");
    const size_t need = nngp::gibbs_stats_workspace_bytes(n, p);
    if (workspace_bytes < need) return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes, need);
    hipError_t e = nngp::gibbs_stats_launch(n, r, Ft, yres, y, X, p, w, noise_w, out, workspace,
                                              (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gibbs_stats launch");
    return NNGP_OK;
}

size_t nngp_row_order_workspace_bytes(int64_t n_rows) { return nngp::row_order_workspace_bytes(n_rows); }

int nngp_row_order(const double* coords, int64_t n_points, int32_t dim, const int32_t* nbr, int32_t m, int64_t i0,
                   int64_t n_rows, int32_t* order, int32_t* nbr_sorted, void* workspace, size_t workspace_bytes,
                   void* stream) {
    if (coords == nullptr || workspace == nullptr) return fail(NNGP_EINVAL, "coords and workspace must be non-null");
    if (dim < 1 || dim > NNGP_MAX_DIM) return fail(NNGP_EUNSUP, "dim=%d outside [1, %d]", dim, NNGP_MAX_DIM);
    if (n_rows < 0 || i0 < 0 || i0 + n_rows > n_points)
        return fail(NNGP_EINVAL, "rows [%lld, %lld) outside [0, %lld)", (long long)i0, (long long)(i0 + n_rows),
                    (long long)n_points);
    if (n_rows > INT32_MAX) return fail(NNGP_EINVAL, "n_rows must be < 2^31");
    if (n_rows > 0 && order == nullptr) return fail(NNGP_EINVAL, "order must be non-null");
    if (m < 0 || m > NNGP_MAX_M) return fail(NNGP_EUNSUP, "m=%d outside [0, %d]", m, NNGP_MAX_M);
    if (nbr_sorted != nullptr && m > 0 && n_rows > 0 && nbr == nullptr)
        return fail(NNGP_EINVAL, "nbr must be non-null when nbr_sorted is requested");
    if (((uintptr_t)workspace & 255) != 0) return fail(NNGP_EINVAL, "workspace must be 256-byte aligned");
    const size_t need = nngp::row_order_workspace_bytes(n_rows);
    if (need == 0 || workspace_bytes < need)
        return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes, need);
    hipError_t e = nngp::row_order_launch(coords, dim, i0, n_rows, order, nbr, m, nbr_sorted, workspace,
                                          workspace_bytes, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "row_order launch");
    return NNGP_OK;
}

size_t nngp_knn_workspace_bytes(int64_t n_points, int32_t dim, int32_t m) {
    (void)m;
    if (n_points < 1 || n_points > INT32_MAX || dim < 1 || dim > NNGP_MAX_DIM) return 0;
    nngp::KnnPlan p;
    if (nngp::knn_plan(n_points, dim, &p) != hipSuccess) return 0;
    return p.total_bytes;
}

static int knn_checks(const double* coords, int64_t n_points, int32_t dim, int32_t m, void* workspace,
                      size_t workspace_bytes, nngp::KnnPlan* plan) {
    if (coords == nullptr || workspace == nullptr) return fail(NNGP_EINVAL, "coords and workspace must be non-null");
    if (n_points < 1 || n_points > INT32_MAX) return fail(NNGP_EINVAL, "n_points=%lld outside [1, 2^31)", (long long)n_points);
    if (dim < 1 || dim > NNGP_MAX_DIM) return fail(NNGP_EUNSUP, "dim=%d outside [1, %d]", dim, NNGP_MAX_DIM);
    if (m < 0 || m > 64) return fail(NNGP_EUNSUP, "m=%d outside [0, 64]", m);
    if (((uintptr_t)workspace & 255) != 0) return fail(NNGP_EINVAL, "workspace must be 256-byte aligned");
    hipError_t e = nngp::knn_plan(n_points, dim, plan);
    if (e != hipSuccess) return hip_fail(e, "knn plan");
    if (workspace_bytes < plan->total_bytes)
        return fail(NNGP_EINVAL, "workspace too small: %zu < %zu bytes", workspace_bytes, plan->total_bytes);
    return NNGP_OK;
}

int nngp_knn_prior(const double* coords, int64_t n_points, int32_t dim, int32_t m, int64_t q0, int64_t q1,
                   int32_t* nbr, void* workspace, size_t workspace_bytes, void* stream) {
    nngp::KnnPlan plan;
    const int rc = knn_checks(coords, n_points, dim, m, workspace, workspace_bytes, &plan);
    if (rc != NNGP_OK) return rc;
    if (q0 < 0 || q1 < q0 || q1 > n_points) return fail(NNGP_EINVAL, "query rows [%lld, %lld) invalid", (long long)q0, (long long)q1);
    if (q1 > q0 && m > 0 && nbr == nullptr) return fail(NNGP_EINVAL, "nbr must be non-null");
    if (q1 == q0 || m == 0) return NNGP_OK;
    hipError_t e = nngp::knn_launch(true, coords, n_points, m, coords, q0, q1, nullptr, nbr, workspace, plan,
                                    (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "knn_prior launch");
    return NNGP_OK;
}

int nngp_knn_prior_rows(const double* coords, int64_t n_points, int32_t dim, int32_t m, const int32_t* rows,
                        int64_t n_rows, int32_t* nbr, void* workspace, size_t workspace_bytes, void* stream) {
    nngp::KnnPlan plan;
    const int rc = knn_checks(coords, n_points, dim, m, workspace, workspace_bytes, &plan);
    if (rc != NNGP_OK) return rc;
    if (n_rows < 0) return fail(NNGP_EINVAL, "n_rows < 0");
    if (n_rows > 0 && m > 0 && (nbr == nullptr || rows == nullptr)) return fail(NNGP_EINVAL, "rows and nbr must be non-null");
    if (n_rows == 0 || m == 0) return NNGP_OK;
    hipError_t e = nngp::knn_launch(true, coords, n_points, m, coords, 0, n_rows, rows, nbr, workspace, plan,
                                    (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "knn_prior_rows launch");
    return NNGP_OK;
}

int nngp_knn_query(const double* ref, int64_t n_ref, int32_t dim, const double* query, int64_t n_query, int32_t k,
                   int32_t* nbr, void* workspace, size_t workspace_bytes, void* stream) {
    nngp::KnnPlan plan;
    const int rc = knn_checks(ref, n_ref, dim, k, workspace, workspace_bytes, &plan);
    if (rc != NNGP_OK) return rc;
    if (n_query < 0) return fail(NNGP_EINVAL, "n_query < 0");
    if (n_query > 0 && k > 0 && (query == nullptr || nbr == nullptr))
        return fail(NNGP_EINVAL, "query and nbr must be non-null");
    if (n_query == 0 || k == 0) return NNGP_OK;
    hipError_t e = nngp::knn_launch(false, ref, n_ref, k, query, 0, n_query, nullptr, nbr, workspace, plan,
                                    (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "knn_query launch");
    return NNGP_OK;
}

}  // extern "C"
