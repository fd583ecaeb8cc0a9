/*
 * nngp.h -- C ABI of libnngp_hip.so, the MI355X (gfx950) NNGP hot path.
 *
 * The reference (bwpriest/pyNNGP) exposes this path only as Python methods of
 * class NNGP; there is no FFI in it.  Each entry point below names the reference
 * interface it replaces (file:line under /root/reference).  The Python binding
 * (pynngp_amd/_lib.py, ctypes) and the torch custom ops (pynngp_amd/ops.py) are
 * thin layers over exactly these symbols; INTEGRATION.md shows the binding a
 * pyNNGP maintainer would add.
 *
 * Conventions
 *   - Every pointer argument except the host-side `partials_host` of
 *     nngp_loglik_from_partials is a DEVICE pointer (hipMalloc / torch CUDA
 *     tensor memory); the caller owns every buffer.
 *   - `stream` is a hipStream_t (NULL = default stream).  All work is
 *     stream-ordered; no call synchronises the host, allocates, or frees.
 *   - Coordinates are fp64 (n_points, dim) row-major, dim = 1, 2 or 3 (the
 *     reference's KDTree takes ordinates of any dimension, nngp.py:55-61); they
 *     must be finite.  Neighbour sets are int32 (rows, m) row-major, padded with -1
 *     (row i holds min(i, m) indices).
 *   - Return 0 on success or a negative NNGP_E* code (nngp_last_error() gives
 *     the message).  Numerical failures are data, not return codes, because the
 *     work is asynchronous: see `partials` of nngp_bf_sweep.
 */
#ifndef NNGP_H
#define NNGP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNGP_OK 0
#define NNGP_EINVAL (-1)    /* bad argument (shape, range, null pointer, small workspace) */
#define NNGP_ENOTPD (-2)    /* a location's C_N / F was not positive definite (nngp_check_partials) */
#define NNGP_EHIP (-3)      /* a HIP runtime call or kernel launch failed */
#define NNGP_EUNSUP (-4)    /* unsupported configuration (e.g. m > 63) */

/* covariance kinds (the reference's `cov` plug-in, nngp.py:6,12), u = phi d: */
#define NNGP_COV_EXPONENTIAL 0 /* sigma2 exp(-u)                                    */
#define NNGP_COV_MATERN32 1    /* sigma2 (1 + u) exp(-u)                            */
#define NNGP_COV_MATERN52 2    /* sigma2 (1 + u + u^2/3) exp(-u)                    */
#define NNGP_COV_GAUSSIAN 3    /* sigma2 exp(-u^2)                                  */
#define NNGP_COV_SPHERICAL 4   /* sigma2 (1 - 3u/2 + u^3/2) for u < 1, else 0       */
#define NNGP_COV_MATERN 5      /* sigma2 u^nu K_nu(u) / (2^(nu-1) Gamma(nu)), 0 < nu <= 50: spNNGP's
                                  "matern" of any smoothness nu (the `nu` argument of the sweeps;
                                  ignored by the other kinds).  m <= 24 (pair kernel) and 25..32
                                  (four-lane kernel): rho from a per-launch table in t = (phi d)^2,
                                  every nu; for nu < 0.9 whose table would pass 160 octaves, below
                                  t = 2^-64 the small-t expansion 1 - A t^nu.  m > 32: the wavefront
                                  kernel's direct Bessel evaluation. */

/* kernels (NNGP_ALGO_AUTO picks the fastest measured one for m, kind and dim); LANE serves 2-D
 * exponential / Matern-3/2 only, QUAD kinds 0..4 in every dimension, PAIRB and WAVE every kind
 * (PAIRB and QUAD: NNGP_COV_MATERN through its table; PAIRB at 25 <= m <= 32: kinds 0..4).  (3 and 7 were comparison-only kernels of earlier
 * builds; they are rejected as unknown.) */
#define NNGP_ALGO_AUTO 0  /* pairb for 1 <= m <= 32 except quad at 31, wave above (matern: see kind 5) */
#define NNGP_ALGO_LANE 1  /* one lane per location (m <= 16)                                 */
#define NNGP_ALGO_WAVE 2  /* one wavefront per location (m <= 63)                            */
#define NNGP_ALGO_QUAD 4  /* four lanes per location (25 <= m <= 32)                         */
#define NNGP_ALGO_PAIRB 5 /* two lanes per location, 2x2-blocked (1 <= m <= 24)              */

/* the kernel NNGP_ALGO_AUTO (or an explicit code, returned as is) resolves to for (m, kind, dim);
 * for NNGP_COV_MATERN the choice depends on nu: nngp_resolve_algo_nu (nngp_resolve_algo assumes a nu
 * the pair kernel's table covers).  nngp_bf_finalize of a matern sweep needs the resolved code. */
int32_t nngp_resolve_algo(int32_t algo, int32_t m, int32_t kind, int32_t dim);
int32_t nngp_resolve_algo_nu(int32_t algo, int32_t m, int32_t kind, int32_t dim, double nu);

#define NNGP_MAX_M 63
#define NNGP_MAX_DIM 3

/* Library version string, e.g. "pynngp_amd 0.3.0 gfx950". */
const char *nngp_version(void);

/* ABI revision of this header (NNGP_ABI_VERSION), for a caller built against an older one to
 * refuse a library whose signatures moved.  Revision 2 (library 0.2.0) changed, relative to 1
 * (0.1.0): nngp_bf_finalize takes workspace_bytes as its 2nd argument; nngp_gibbs_w_sweep reads
 * (n, 4) member rows (nngp_gibbs_member_rows) and lost its `off` argument; nngp_bf_sweep /
 * nngp_bf_cross take `nu` after tau2; nngp_bf_sweep_blocks serves 1 <= m <= 32.  Revision 3
 * (library 0.3.0) adds the tile pair plans (nngp_pair_plan_*, nngp_bf_sweep_plan), the batched
 * chains' sweeps (nngp_gibbs_w_sweep_chains, _il) and the device colouring (nngp_color_moral_graph_dev);
 * NNGP_ALGO_AUTO / PAIRB / QUAD take the general Matern kind for every nu; nothing earlier moved.
 * Revision 4 (library 0.4.0): the pair plans are per wave (a new plan format, m <= 17) and their info
 * array holds 10 words (NNGP_PLAN_INFO_LEN: + the nbr / order pointers, checked by nngp_bf_sweep_plan). */
#define NNGP_ABI_VERSION 4
int32_t nngp_abi_version(void);

/* Message for the last error returned on the calling thread. */
const char *nngp_last_error(void);

/* ---------------------------------------------------------------------------
 * Neighbour sets.
 * Replaces NNGP._make_s_neighbor_sets, pyNNGP/nngp.py:49-62 (a sklearn KDTree
 * rebuilt on s[0:i] for every i; ordering key sklearn euclidean_rdist64,
 * sklearn/metrics/_dist_metrics.pxd:26-40).
 * For every query row i in [q0, q1): the k = min(m, i) nearest points among
 * coords[0:i], ascending fp64 rdist = (0 + t0*t0) + t1*t1 (no FMA), exact
 * ties by lower index, written to nbr[(i - q0) * m + s], s < k; -1 beyond.  rdist
 * sums t_k^2 over the dim coordinates in axis order, unfused, as sklearn does.
 * Requires n_points <= INT32_MAX, 1 <= dim <= 3, 0 <= m <= 64,
 * 0 <= q0 <= q1 <= n_points, and finite coordinates (NaN / inf give unspecified
 * sets; the Python layer rejects them).
 * ------------------------------------------------------------------------- */
size_t nngp_knn_workspace_bytes(int64_t n_points, int32_t dim, int32_t m);
int nngp_knn_prior(const double *coords, int64_t n_points, int32_t dim, int32_t m, int64_t q0, int64_t q1,
                   int32_t *nbr, void *workspace, size_t workspace_bytes, void *stream);

/* Same neighbour sets for an arbitrary list of locations: query row t is point rows[t]
 * (its min(m, rows[t]) nearest among coords[0:rows[t]]), written to nbr[t * m + s].
 * Used to build a shard's sets when the shard is a range of a spatial storage order
 * (pynngp_amd.sweep.ShardedLogLik, layout "storage").  Workspace as nngp_knn_prior. */
int nngp_knn_prior_rows(const double *coords, int64_t n_points, int32_t dim, int32_t m, const int32_t *rows,
                        int64_t n_rows, int32_t *nbr, void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Unrestricted k-nearest neighbours of query points among a reference set.
 * Replaces the sklearn searches behind NNGP._init_ws (pyNNGP/nngp.py:45-47,
 * KNeighborsRegressor(n_neighbors=5).fit(t, y).predict(s)) and
 * NNGP._make_t_neighbor_sets (nngp.py:64-71, KDTree(s).query(t, m)).
 * nbr[q * k + s] = index into ref of the s-th nearest point to query[q]
 * ((rdist, index) order, self included when a query point is in ref), -1 for
 * s >= n_ref.  ref and query are (n, dim).  Workspace: nngp_knn_workspace_bytes(n_ref, dim, k).
 * ------------------------------------------------------------------------- */
int nngp_knn_query(const double *ref, int64_t n_ref, int32_t dim, const double *query, int64_t n_query, int32_t k,
                   int32_t *nbr, void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Fused B/F + log-likelihood sweep over locations i0 .. i0 + n_rows - 1.
 * Replaces the per-location stubs of class NNGP:
 *   _CNs  nngp.py:78-82   C_{N(s_i)}       (covariance among the neighbours, + tau2 I)
 *   _Ccross nngp.py:84-86 C_{s_i, N(s_i)}  (location vs neighbours)
 *   _Cs   nngp.py:92-96   C_{s_i, s_i}     (sigma2 + tau2)
 *   _Bsi  nngp.py:73-76   B_i = C_{s_i,N} C_N^{-1}       -> B (n_rows, m), 0 in -1 slots
 *   _Fsi  nngp.py:88-90   F_i = C_ii - B_i C_{N,s_i}     -> F (n_rows,)
 * and the log-likelihood sweep consumed by oneSample (nngp.py:98-101, absent):
 *   partials[0] = sum_i log F_i
 *   partials[1] = sum_i (v_i - B_i v_N(i))^2 / F_i        (0 when values == NULL)
 *   partials[2] = first location index whose Cholesky pivot or F_i is not > 0, else -1
 *   partials[3] = first location index with an invalid neighbour index (>= n_points, or
 *                 negative other than the -1 padding), else -1; such a row's slot is
 *                 decoupled (a far-away point), so its B / F / log-lik terms are finite but
 *                 meaningless: callers check the flag (nngp_check_partials)
 *   log-lik = -1/2 (n_rows log 2 pi + partials[0] + partials[1]).
 * Rows flagged in partials[2] get B = F = NaN.  The sum order is fixed, so the
 * partials are bit-reproducible run to run.
 * coords: (n_points, dim); nbr: (n_rows, m); order: NULL (row t of nbr is location
 * i0 + t) or the nngp_row_order layout (row t of nbr is location i0 + order[t],
 * i.e. pass nbr_sorted); values: (n_points,) or NULL;
 * B, F: may be NULL (log-lik only); R: NULL or (n_rows,) residuals
 * r_i = v_i - B_i v_N(i) (needs values; the Gibbs w-update keeps them current);
 * partials: 4 doubles, or NULL to defer the final fold: the per-block records stay in
 * the workspace and nngp_bf_finalize (same n_rows, m, kind, dim, algo) folds them later,
 * e.g. on another stream while the next sweep (with another workspace) runs.
 * workspace: nngp_bf_sweep_workspace_bytes(n_rows, m, kind, dim, algo) bytes, 256-B aligned, its first
 * 256 bytes zeroed once before the first sweep that uses it (the pair kernel's header: its tile count
 * and the ticket of the fold a small sweep does in its last block, which every sweep leaves at zero;
 * the same holds for nngp_bf_cross and nngp_bf_sweep_blocks workspaces).
 * kind, sigma2 > 0, phi > 0, tau2 >= 0: the covariance (the reference's `cov`); nu: the smoothness
 * of NNGP_COV_MATERN (0 < nu <= 50), ignored by the other kinds.
 * ------------------------------------------------------------------------- */
size_t nngp_bf_sweep_workspace_bytes(int64_t n_rows, int32_t m, int32_t kind, int32_t dim, int32_t algo);
int nngp_bf_sweep(const double *coords, int64_t n_points, int32_t dim, const int32_t *nbr, const int32_t *order,
                  int64_t n_rows, int32_t m, int64_t i0, int32_t kind, double sigma2, double phi, double tau2,
                  double nu, const double *values, double *B, double *F, double *R, double *partials, void *workspace,
                  size_t workspace_bytes, int32_t algo, void *stream);
/* The deferred fold of a sweep run with partials == NULL (fixed order: the same
 * bits as the in-line fold).  n_rows, m, kind, dim and algo must be the sweep's (they select
 * the kernel, hence the record layout); workspace_bytes is checked against the size that
 * sweep needed, so a mismatched call fails with NNGP_EINVAL instead of reading past it. */
int nngp_bf_finalize(const void *workspace, size_t workspace_bytes, int64_t n_rows, int32_t m, int32_t kind,
                     int32_t dim, int32_t algo, double *partials, void *stream);

/* ---------------------------------------------------------------------------
 * Wave pair plans: the same sweep with every covariance a wavefront's locations share evaluated once.
 * The pair kernel (NNGP_ALGO_PAIRB) sweeps 32 consecutive rows per wavefront; in a spatial visiting
 * order neighbouring locations share most of their neighbours, so only ~46 % of a wave's joint-block
 * entries are distinct point pairs (N = 1e6, m = 15).  A plan -- built once per (nbr, order, i0,
 * n_points), like the neighbour sets -- lists per wave its distinct points and pairs and, per lane,
 * where each of its joint-block entries lives; nngp_bf_sweep_plan then evaluates each pair once into
 * the wave's LDS slice and factors every location's block from there.  Same reference methods as
 * nngp_bf_sweep (_CNs / _Ccross / _Cs / _Bsi / _Fsi, nngp.py:73-96); its B, F, R are bit-identical to
 * nngp_bf_sweep's with NNGP_ALGO_PAIRB on the same arguments, and so are its partials (tiles whose
 * waves exceed the LDS budget are swept by the unplanned kernel into the same records).
 * nngp_pair_plan_supported: 1 when plans serve (m, kind, dim): 2 <= m <= 17, kinds 0..4, dim 1..3.
 * nngp_pair_plan_bytes: the plan buffer's size (0: unsupported m).
 * nngp_pair_plan_build: builds the plan for the sweep's nbr / order / i0 / n_points (device
 * pointers as nngp_bf_sweep; 256-B aligned plan) on `stream`, then SYNCHRONISES the stream (a setup
 * call, the one exception to the no-synchronisation rule above) to fill the host array
 * info[NNGP_PLAN_INFO_LEN]: tiles swept through the plan, tiles swept directly, the geometry the
 * plan was built for (n_rows, m, dim, i0, n_points), a tag, and the nbr and order pointers.
 * nngp_bf_sweep_plan: nngp_bf_sweep's arguments (algo PAIRB implied; kinds 0..4, no nu) plus the
 * plan and its info; n_rows, m, dim, i0, n_points and the nbr / order pointers must be those in info
 * (checked: NNGP_EINVAL).  The plan is stale once the contents of nbr or order change: the kernel
 * re-derives a per-location checksum of the words it reads and flags a mismatching location in
 * partials[3] with B = F = R = NaN, so a stale plan never returns the old neighbour sets' results.
 * ------------------------------------------------------------------------- */
#define NNGP_PLAN_INFO_LEN 10
int nngp_pair_plan_supported(int32_t m, int32_t kind, int32_t dim);
size_t nngp_pair_plan_bytes(int64_t n_rows, int32_t m, int32_t dim);
int nngp_pair_plan_build(const int32_t *nbr, const int32_t *order, int64_t n_rows, int32_t m, int64_t i0,
                         int64_t n_points, int32_t dim, void *plan, size_t plan_bytes, int64_t *info, void *stream);
int nngp_bf_sweep_plan(const double *coords, int64_t n_points, int32_t dim, const int32_t *nbr, const int32_t *order,
                       int64_t n_rows, int32_t m, int64_t i0, int32_t kind, double sigma2, double phi, double tau2,
                       const double *values, double *B, double *F, double *R, double *partials, void *workspace,
                       size_t workspace_bytes, const void *plan, size_t plan_bytes, const int64_t *info,
                       void *stream);

/* ---------------------------------------------------------------------------
 * B/F of query locations t against a reference set S (prediction / kriging at
 * t not in S).  SURVEY.md 8(f) row 2: the reference builds Nt for refType != 'S=T'
 * (NNGP._make_t_neighbor_sets, pyNNGP/nngp.py:64-71, KDTree(s).query(t, m)) but
 * never evaluates B_t / F_t; this is the same fused kernel as nngp_bf_sweep with
 * the location row taken from `query`:
 *   C_N = C(S_N) + tau2 I over the neighbours nbr[(q - q0) * m + k] (indices into
 *   ref; any of them, no prior restriction; -1 = unused slot), c = C(t_q, S_N),
 *   C_tt = sigma2 + tau2, B_t = c^T C_N^{-1}, F_t = C_tt - c^T C_N^{-1} c.
 * ref_values (nullable): v on S.  query_values (nullable; needs ref_values): v at t.
 * R[q] = query_values[q] - B_t v_N(t) (query_values NULL: 0 - B_t v_N(t), i.e. minus
 * the kriging mean).  partials as nngp_bf_sweep (with query_values: the
 * conditional log density of v_t given v_S).  Rows q in [q0, q0 + n_rows) of
 * n_query; order / workspace as nngp_bf_sweep (nngp_row_order on the query
 * coordinates; nngp_bf_sweep_workspace_bytes), kind / theta / nu as nngp_bf_sweep.  ref and
 * query are (n, dim).
 * ------------------------------------------------------------------------- */
int nngp_bf_cross(const double *ref, int64_t n_ref, int32_t dim, const double *query, int64_t n_query,
                  const int32_t *nbr, const int32_t *order, int64_t n_rows, int32_t m, int64_t q0, int32_t kind,
                  double sigma2, double phi, double tau2, double nu, const double *ref_values,
                  const double *query_values,
                  double *B, double *F, double *R, double *partials, void *workspace, size_t workspace_bytes,
                  int32_t algo, void *stream);

/* ---------------------------------------------------------------------------
 * A covariance of the caller's own (the reference's `cov` is an arbitrary plug-in,
 * pyNNGP/nngp.py:6,12, called on coordinate rows at :82,:96; SURVEY.md 8(b) asks for callables):
 * the caller evaluates its function on every joint block -- an isotropic function of
 * nngp_joint_dist's distances, or any cov(a, b) on the blocks' gathered coordinates -- and the
 * blocks drive the same fused sweep.
 * nngp_joint_dist: for nbr row t (location i = i0 + (order ? order[t] : t); joint rows
 *   a = 0..m-1 the neighbour slots, row m the location, from qcoords) the packed lower
 *   triangle of the joint block's distances, entry (a, b), b <= a, at
 *   dist[(a (a + 1) / 2 + b) * n_rows + t] -- nngp_joint_entries(m) = (m+1)(m+2)/2 entries
 *   per row, entry-major; 0 on the diagonal, +inf where a slot holds no point.  Distances are
 *   sqrt of the unfused sum of squared coordinate differences.
 * nngp_bf_sweep_blocks: the fused B/F + log-lik sweep (outputs, partials, order and values
 *   as nngp_bf_sweep / nngp_bf_cross: values (n_points,) of the neighbours, qvalues (n_locs,)
 *   of the locations, may be NULL) with the joint blocks' covariances read from `cov` in that
 *   layout -- cov[e] = C(dist[e]) plus the nugget on the diagonal entries; entries of slots
 *   without a point are ignored (decoupled exactly).  1 <= m <= 32 (the two-lane blocked
 *   kernel up to 24, the four-lane kernel for 25..32); workspace
 *   nngp_bf_sweep_blocks_workspace_bytes(n_rows), 256-B aligned; partials required.
 * ------------------------------------------------------------------------- */
/* out[k] = u^nu K_nu(u) / (2^(nu-1) Gamma(nu)) for n arguments u >= 0 (the Matern correlation
 * of NNGP_COV_MATERN, elementwise; 0 < nu <= 50): a building block for such covariances. */
int nngp_matern_eval(const double *u, int64_t n, double nu, double *out, void *stream);
int64_t nngp_joint_entries(int32_t m);
int nngp_joint_dist(const double *coords, int64_t n_points, int32_t dim, const double *qcoords, int64_t n_locs,
                    const int32_t *nbr, const int32_t *order, int64_t n_rows, int32_t m, int64_t i0, double *dist,
                    void *stream);
size_t nngp_bf_sweep_blocks_workspace_bytes(int64_t n_rows);
int nngp_bf_sweep_blocks(const double *cov, const int32_t *nbr, const int32_t *order, int64_t n_points, int64_t n_rows,
                         int32_t m, int64_t i0, int64_t n_locs, const double *values, const double *qvalues, double *B,
                         double *F, double *R, double *partials, void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Visiting order for nngp_bf_sweep (a speed option; no reference counterpart:
 * the reference visits locations in input order, nngp.py:51).
 * order[t] = the t-th local row (0 .. n_rows-1) of locations i0 .. i0+n_rows-1
 * in Z-order of their coordinates, ties by row; if nbr_sorted is non-NULL it
 * receives nbr's rows in that order (nbr_sorted[t] = nbr[order[t]], (n_rows, m)).
 * Passing (nbr_sorted, order) to nngp_bf_sweep keeps each block's / XCD's
 * neighbour gathers spatially compact (L2 hits) and its index reads coalesced;
 * B and F are bit-identical with or without it (still written at their natural
 * rows), the partials' summation order follows it.
 * Workspace: nngp_row_order_workspace_bytes(n_rows).
 * ------------------------------------------------------------------------- */
size_t nngp_row_order_workspace_bytes(int64_t n_rows);
int nngp_row_order(const double *coords, int64_t n_points, int32_t dim, const int32_t *nbr, int32_t m, int64_t i0,
                   int64_t n_rows, int32_t *order, int32_t *nbr_sorted, void *workspace, size_t workspace_bytes,
                   void *stream);

/* ---------------------------------------------------------------------------
 * Multi-GPU: fold the all-gathered partials of `world` ranks (device array
 * (world, 4), rank-major, e.g. from an RCCL all-gather) in rank order:
 * partials[0..1] = sums, partials[2..3] = smallest non-negative flag or -1.
 * Every rank gets the bit-identical result.  No reference counterpart (the
 * reference is single-process).
 * nngp_combine_partials_batch: the same fold for n_slots independent sweeps exchanged in ONE
 * all-gather: gathered (world, n_slots, 4) rank-major (each rank contributed its (n_slots, 4)
 * block), partials (n_slots, 4); slot k's result is bit-identical to nngp_combine_partials of
 * that sweep alone.
 * ------------------------------------------------------------------------- */
int nngp_combine_partials(const double *gathered, int32_t world, double *partials, void *stream);
int nngp_combine_partials_batch(const double *gathered, int32_t world, int64_t n_slots, double *partials,
                                void *stream);

/* ---------------------------------------------------------------------------
 * Gibbs sampler for the response model y = X beta + w + eps (SURVEY.md 8(f)
 * row 1).  Replaces NNGP.oneSample, nngp.py:98-101, whose update_wt / update_ws /
 * update_y_unobserved do not exist in the reference; model of Datta et al. 2016
 * as named by the reference docstrings.  Whole-field (single-GPU) arrays.
 *
 * nngp_reverse_neighbors: CSR transpose of nbr (n, m): for location i the
 *   entries e in [off[i], off[i+1]) list the rows j = rev_j[e] whose neighbour
 *   slot rev_k[e] is i, ascending j.  off: n+1, rev_j / rev_k: n*m ints (device).
 * nngp_color_moral_graph (HOST pointers, host computation): greedy colouring
 *   of the moral graph (i ~ N(i); co-parents of a child ~ each other) in index
 *   order; returns the number of colours (or a negative NNGP_E* code).
 * nngp_color_moral_graph_dev: the same colouring (bit for bit: node i takes the smallest colour
 *   no moral neighbour k < i holds) on the device, in parallel rounds (nbr, off, rev_j, color:
 *   device; workspace: >= 256 device bytes); a setup call that synchronises the stream once per 16
 *   rounds.  Returns the number of colours, or a negative NNGP_E* code (NNGP_EUNSUP past 256
 *   colours: use the host version).
 * nngp_gibbs_prepare: fold the factors of the unit-variance field (sigma2 = 1,
 *   tau2 = 0; B (n, m) and Ft (n,) from nngp_bf_sweep) into reverse-list order for
 *   the w sweeps: B_{j,i} and B_{j,i}/F_j per reverse entry, sum_e B_{j,i}^2/F_j and
 *   1/F_i per location, into `prep` (device, nngp_gibbs_prep_bytes(n, m) bytes,
 *   256-B aligned).  Call it again whenever B / Ft change (a new phi accepted).
 *   order: unused (accepted for compatibility; the preparation streams the reverse
 *   lists in their own order).
 * nngp_gibbs_member_rows: member_rows[g] = (members[g], off[members[g]], off[members[g] + 1], 0)
 *   (device int32 (n, 4), 16-B aligned) for `members` (device), the locations grouped by
 *   colour -- built once per colouring; the colour steps then start with one coalesced
 *   16-B load per member instead of two dependent loads.
 * nngp_gibbs_w_sweep: one sweep of w_i | rest over the colours in order;
 *   `member_rows` (nngp_gibbs_member_rows) lists the locations grouped by colour,
 *   color_off_host (host, n_colors + 1) delimits them.  r (n,) holds the residuals
 *   w_i - B_i w_N(i) (nngp_bf_sweep's R), kept current in place with w.
 *   yres = y - X beta.  noise_w: NULL (homoscedastic noise, variance tau2) or n
 *   positive weights h_i, the noise variance of location i being tau2 / h_i (e.g.
 *   h_i = 1 / eps_i^2 for the reference's per-point measurement sigmas, nngp.py:9).
 *   z: NULL (Philox4x32-10 normals keyed by seed, counter
 *   (location, sweep)) or n given standard normals (for testing).
 * nngp_gibbs_normals: z[i] = the Philox4x32-10 normal the sweep would draw for
 *   (seed, location i, sweep), for all n locations in one parallel pass; passing it
 *   as nngp_gibbs_w_sweep's z gives the bit-identical chain with shorter colour steps.
 * nngp_gibbs_w_sweep_chains: nngp_gibbs_w_sweep for `chains` (1..8) independent chains of the same
 *   field -- the same member_rows / colours / rev_j / noise_w, each chain c its own prep[c] (its
 *   phi's factors), sigma2[c], tau2[c] (host arrays), yres[c], w[c], r[c] and given normals z[c]
 *   (host arrays of device pointers) -- in ONE launch per colour; chain c's result is bit-identical
 *   to nngp_gibbs_w_sweep on its own arguments (with z given).
 * nngp_gibbs_w_sweep_chains_il: the same with every chain's w and r interleaved in two (n, chains)
 *   row-major, 16-byte aligned arrays (chain c of location i at [i * chains + c]): a child's r_j of all chains is one
 *   contiguous run, so the colour steps' scattered accesses move one sector for all chains; the
 *   results are the per-chain call's, bit for bit.
 * nngp_gibbs_stats: out[0] = sum r_i^2 / Ft_i, out[1] = sum h_i (yres_i - w_i)^2,
 *   out[2 + c] = sum_i h_i X[i, c] (y_i - w_i) for c < p (X row-major (n, p));
 *   h_i = noise_w[i], or 1 when noise_w is NULL.
 *
 * One chain sharded over ranks (the w sweep's per-colour exchange;
 * pynngp_amd.gibbs.ShardedSeqNNGP): rank r owns the storage rows [row0, row1) and keeps
 * replicas of w and r, exact on its own rows, their out-of-shard children (halo) and the
 * parents of both.
 * nngp_gibbs_prepare_range: nngp_gibbs_prepare for the rows [row0, row1) only (their
 *   reverse entries [off[row0], off[row1]), P and 1/F); B / Ft must be current on those
 *   rows and their children.  The full range is nngp_gibbs_prepare.
 * nngp_gibbs_w_color: ONE colour step over member_rows (n_members rows of
 *   nngp_gibbs_member_rows, e.g. the run of one colour this rank owns), arguments as
 *   nngp_gibbs_w_sweep; w_out (NULL or n_members doubles) receives each member's new
 *   w, the values the other ranks replay.
 * nngp_gibbs_w_color_dev: the same step with (sigma2, tau2) read from device memory
 *   var[0], var[1] (the kernel forms 1/var exactly as the host would: the same bits) and
 *   the given normals z (required) -- launch arguments that stay fixed across iterations,
 *   so a captured HIP graph of the colour loop replays with each iteration's values.
 * nngp_gibbs_w_apply: replay other ranks' draws of one colour: rows (device int32
 *   (n_rows, 4), 16-B aligned) = (location i, off[i], off[i + 1], src); w_src[src] is the
 *   owner's new w_i.  dw = w_src[src] - w[i] (this rank's replica: the owner's operands),
 *   w[i] = w_src[src], r[i] += dw, r[j] -= B[j, rev_k[e]] dw over the children -- the
 *   owner's arithmetic, so every replica stays bit-identical to the owner's values.
 * ------------------------------------------------------------------------- */
size_t nngp_reverse_workspace_bytes(int64_t n, int32_t m);
int nngp_reverse_neighbors(const int32_t *nbr, int64_t n, int32_t m, int32_t *off, int32_t *rev_j, int32_t *rev_k,
                           void *workspace, size_t workspace_bytes, void *stream);
int64_t nngp_color_moral_graph(const int32_t *nbr_host, const int32_t *off_host, const int32_t *rev_j_host,
                               int64_t n, int32_t m, int32_t *color_host);
int64_t nngp_color_moral_graph_dev(const int32_t *nbr, const int32_t *off, const int32_t *rev_j, int64_t n, int32_t m,
                                   int32_t *color, void *workspace, size_t workspace_bytes, void *stream);
size_t nngp_gibbs_prep_bytes(int64_t n, int32_t m);
int nngp_gibbs_prepare(const double *B, const double *Ft, const int32_t *off, const int32_t *rev_j,
                       const int32_t *rev_k, const int32_t *order, int64_t n, int32_t m, void *prep,
                       size_t prep_bytes, void *stream);
int nngp_gibbs_member_rows(const int32_t *members, int64_t n, const int32_t *off, int32_t *member_rows, void *stream);
int nngp_gibbs_w_sweep(const int32_t *member_rows, const int32_t *color_off_host, int32_t n_colors, const void *prep,
                       int64_t n, int32_t m, double sigma2, double tau2, const double *yres, const double *noise_w,
                       double *w, double *r, const int32_t *rev_j, const double *z, uint64_t seed, uint64_t sweep,
                       void *stream);
/* nngp_gibbs_w_sweep_tiles: the same w sweep, tiled (pynngp_amd/gibbs_tiles.py builds the plan): one launch
 *   per phase, one workgroup per tile of the phase holding its footprint's r and its rows' new w in LDS and
 *   running every colour of its rows in order, in steps; the tiles of a phase have disjoint footprints (each
 *   node and its children), so the sweep is a valid colour sweep in the plan's (level, phase, colour) order.
 *   The plan is contiguous: the storage order is the plan's node order.
 *   tiles: the tile ids of every phase, phase p's at [phase_off_host[p], phase_off_host[p + 1]) (host
 *   offsets); phase_lds_host[p]: its dynamic LDS bytes (gibbs_tiles.tile_lds_bytes of its largest tile);
 *   tinfo (n_tiles, 8) int32, 16-byte aligned: the tile's rows [n0, n1), its footprint range [f0, f1) in
 *   tfp, its step range [s0, s1) in tstep, two zeros; tstep: each step's first row (tile-local), a step
 *   being <= 64 rows of one colour with <= ecap reverse entries (ecap <= 2048); tfp: each tile's footprint
 *   (its rows first, then the halo); rev_loc (n_entries): the footprint-local index of reverse entry e's
 *   child; off: the reverse lists' offsets, n_entries = off[n]; z: the normals (nngp_gibbs_normals).
 *   Round 6. */
int nngp_gibbs_w_sweep_tiles(const int32_t *tiles, const int32_t *phase_off_host, const int32_t *phase_lds_host,
                             int32_t n_phases, const int32_t *tinfo, const int32_t *tstep, int32_t ecap,
                             const int32_t *tfp, const int32_t *off, const int32_t *rev_loc, const void *prep,
                             int64_t n, int32_t m, int64_t n_entries, double sigma2, double tau2, const double *yres,
                             const double *noise_w, double *w, double *r, const double *z, void *stream);
int nngp_gibbs_w_sweep_chains(const int32_t *member_rows, const int32_t *color_off_host, int32_t n_colors,
                              int32_t chains, const void *const *prep, int64_t n, int32_t m, const double *sigma2,
                              const double *tau2, const double *const *yres, const double *noise_w, double *const *w,
                              double *const *r, const int32_t *rev_j, const double *const *z, void *stream);
int nngp_gibbs_w_sweep_chains_il(const int32_t *member_rows, const int32_t *color_off_host, int32_t n_colors,
                                 int32_t chains, const void *const *prep, int64_t n, int32_t m, const double *sigma2,
                                 const double *tau2, const double *const *yres, const double *noise_w, double *w_il,
                                 double *r_il, const int32_t *rev_j, const double *const *z, void *stream);
int nngp_gibbs_normals(int64_t n, uint64_t seed, uint64_t sweep, double *z, void *stream);
int nngp_gibbs_prepare_range(const double *B, const double *Ft, const int32_t *off, const int32_t *rev_j,
                             const int32_t *rev_k, int64_t n, int32_t m, int64_t row0, int64_t row1, void *prep,
                             size_t prep_bytes, void *stream);
int nngp_gibbs_w_color(const int32_t *member_rows, int64_t n_members, const void *prep, int64_t n, int32_t m,
                       double sigma2, double tau2, const double *yres, const double *noise_w, double *w, double *r,
                       const int32_t *rev_j, const double *z, uint64_t seed, uint64_t sweep, double *w_out,
                       void *stream);
int nngp_gibbs_w_color_dev(const int32_t *member_rows, int64_t n_members, const void *prep, int64_t n, int32_t m,
                           const double *var, const double *yres, const double *noise_w, double *w, double *r,
                           const int32_t *rev_j, const double *z, double *w_out, void *stream);
int nngp_gibbs_w_apply(const int32_t *rows, int64_t n_rows, const double *w_src, const double *B, int64_t n, int32_t m,
                       double *w, double *r, const int32_t *rev_j, const int32_t *rev_k, void *stream);
size_t nngp_gibbs_stats_workspace_bytes(int64_t n, int32_t p);
int nngp_gibbs_stats(int64_t n, const double *r, const double *Ft, const double *yres, const double *y,
                     const double *X, int32_t p, const double *w, const double *noise_w, double *out,
                     void *workspace, size_t workspace_bytes, void *stream);

/* Host helper for callers that synchronise ("-2 means a non-positive
 * pivot; report the first bad index through an out-param"): given host-resident
 * partials of a finished sweep, returns NNGP_OK, NNGP_ENOTPD with *first_bad_row = the
 * first location whose pivot / F was not > 0, or NNGP_EINVAL with *first_bad_index = the
 * first location with an out-of-range neighbour index (either out-param may be NULL;
 * -1 when not applicable). */
int nngp_check_partials(const double *partials_host, int64_t *first_bad_row, int64_t *first_bad_index);

/* Host helper: -1/2 (n_rows log 2 pi + p[0] + p[1]) from host-resident partials. */
double nngp_loglik_from_partials(const double *partials_host, int64_t n_rows);

#ifdef __cplusplus
}
#endif
#endif /* NNGP_H */
