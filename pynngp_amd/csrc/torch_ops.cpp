// PyTorch-ROCm operators over the C ABI of libnngp_hip.so: TORCH_LIBRARY(nngp, ...).
//
// The drop-in boundary the north_star names ("exposed to Python as a PyTorch-ROCm custom
// op so the SeqNNGP fit/sample surface is a drop-in") as a native op library: the
// schemas are registered with the dispatcher here, the CUDA (= HIP on ROCm; PyTorch's
// key name, not a compat layer) implementations call include/nngp.h directly on torch's
// current HIP stream, so a call from Python is one dispatcher hop into C++ -- no ctypes,
// no Python in between.  CPU tensors have no kernel registered: they raise (there is no
// CPU fallback).  pynngp_amd/ops.py loads this library and adds the fake (meta) kernels
// for tracing; pynngp_amd.sweep.ShardedLogLik and pynngp_amd.gibbs.SeqNNGP sweep through
// nngp::bf_sweep_out.
//
// Reference interfaces replaced (pyNNGP, /root/reference): knn_prior(_rows) <-
// NNGP._make_s_neighbor_sets nngp.py:49-62; knn_query <- _init_ws / _make_t_neighbor_sets
// nngp.py:45-47,64-71; bf_sweep(_out) <- _CNs/_Ccross/_Cs/_Bsi/_Fsi nngp.py:73-96 and the
// log-likelihood oneSample needs (nngp.py:98-101); bf_cross <- B_t / F_t at t not in S.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "../../include/nngp.h"

namespace {

// Every op runs on the current stream of ITS TENSORS' device, under a device guard for that
// device (a tensor on cuda:1 while cuda:0 is current must not launch on cuda:0's stream).
void* stream(const at::Tensor& t) { return (void*)at::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_rc(int rc, const char* what) { TORCH_CHECK(rc == NNGP_OK, what, " failed (", rc, "): ", nngp_last_error()); }

void check_coords(const at::Tensor& c, const char* name) {
    TORCH_CHECK(c.is_cuda(), name, " must be a ROCm GPU tensor (there is no CPU fallback)");
    TORCH_CHECK(c.scalar_type() == at::kDouble && c.dim() == 2 && c.size(1) >= 1 && c.size(1) <= NNGP_MAX_DIM,
                name, " must be float64 (N, dim), 1 <= dim <= ", NNGP_MAX_DIM);
    TORCH_CHECK(c.is_contiguous(), name, " must be contiguous");
}

void check_same_device(const at::Tensor& a, const at::Tensor& b, const char* name) {
    TORCH_CHECK(b.device() == a.device(), name, " is on ", b.device(), ", expected ", a.device());
}

void check_f64(const c10::optional<at::Tensor>& t, at::IntArrayRef shape, const at::Tensor& like, const char* name) {
    if (!t.has_value()) return;
    TORCH_CHECK(t->scalar_type() == at::kDouble && t->sizes() == shape && t->is_contiguous(), name,
                " must be a contiguous float64 tensor of shape ", shape);
    check_same_device(like, *t, name);
}

void check_nbr(const at::Tensor& nbr, const at::Tensor& like) {
    TORCH_CHECK(nbr.scalar_type() == at::kInt && nbr.dim() == 2 && nbr.is_contiguous(),
                "nbr must be a contiguous int32 (rows, m) tensor");
    check_same_device(like, nbr, "nbr");
}

template <typename T>
T* ptr(const c10::optional<at::Tensor>& t) {
    return t.has_value() ? (T*)t->data_ptr() : nullptr;
}

// a sweep workspace's first 256 bytes (the pair kernel's header: tile count, fused-fold ticket) start at
// zero (include/nngp.h); the rest is scratch
at::Tensor workspace(int64_t bytes, const at::Tensor& like) {
    auto ws = at::empty({bytes > 256 ? bytes : 256}, like.options().dtype(at::kByte));
    ws.narrow(0, 0, 256).zero_();
    return ws;
}

// ---------------------------------------------------------------- neighbour sets
at::Tensor knn_prior(const at::Tensor& coords, int64_t m, int64_t q0, int64_t q1) {
    check_coords(coords, "coords");
    const at::OptionalDeviceGuard guard(coords.device());
    const int64_t n = coords.size(0), d = coords.size(1);
    TORCH_CHECK(0 <= q0 && q0 <= q1 && q1 <= n, "query rows [", q0, ", ", q1, ") outside [0, ", n, ")");
    auto out = at::empty({q1 - q0, m}, coords.options().dtype(at::kInt));
    auto ws = workspace((int64_t)nngp_knn_workspace_bytes(n, (int32_t)d, (int32_t)m), coords);
    check_rc(nngp_knn_prior(coords.data_ptr<double>(), n, (int32_t)d, (int32_t)m, q0, q1, out.data_ptr<int32_t>(),
                            ws.data_ptr(), ws.numel(), stream(coords)),
             "nngp_knn_prior");
    return out;
}

at::Tensor knn_prior_rows(const at::Tensor& coords, int64_t m, const at::Tensor& rows) {
    check_coords(coords, "coords");
    const at::OptionalDeviceGuard guard(coords.device());
    TORCH_CHECK(rows.scalar_type() == at::kInt && rows.dim() == 1 && rows.is_contiguous(), "rows must be int32 (n_rows,)");
    check_same_device(coords, rows, "rows");
    const int64_t n = coords.size(0), d = coords.size(1);
    auto out = at::empty({rows.size(0), m}, coords.options().dtype(at::kInt));
    auto ws = workspace((int64_t)nngp_knn_workspace_bytes(n, (int32_t)d, (int32_t)m), coords);
    check_rc(nngp_knn_prior_rows(coords.data_ptr<double>(), n, (int32_t)d, (int32_t)m, rows.data_ptr<int32_t>(),
                                 rows.size(0), out.data_ptr<int32_t>(), ws.data_ptr(), ws.numel(), stream(coords)),
             "nngp_knn_prior_rows");
    return out;
}

at::Tensor knn_query(const at::Tensor& ref, const at::Tensor& query, int64_t k) {
    check_coords(ref, "ref");
    const at::OptionalDeviceGuard guard(ref.device());
    check_coords(query, "query");
    check_same_device(ref, query, "query");
    TORCH_CHECK(ref.size(1) == query.size(1), "ref and query have different dimensions");
    const int64_t d = ref.size(1);
    auto out = at::empty({query.size(0), k}, ref.options().dtype(at::kInt));
    auto ws = workspace((int64_t)nngp_knn_workspace_bytes(ref.size(0), (int32_t)d, (int32_t)k), ref);
    check_rc(nngp_knn_query(ref.data_ptr<double>(), ref.size(0), (int32_t)d, query.data_ptr<double>(), query.size(0),
                            (int32_t)k, out.data_ptr<int32_t>(), ws.data_ptr(), ws.numel(), stream(ref)),
             "nngp_knn_query");
    return out;
}

// ---------------------------------------------------------------- the fused sweep
// out-variant: every output buffer is the caller's (the hot path: no allocation per sweep)
void bf_sweep_out(const at::Tensor& coords, const at::Tensor& nbr, const c10::optional<at::Tensor>& order, int64_t i0,
                  int64_t kind, double sigma2, double phi, double tau2, const c10::optional<at::Tensor>& values,
                  const c10::optional<at::Tensor>& B, const c10::optional<at::Tensor>& F,
                  const c10::optional<at::Tensor>& R, const at::Tensor& partials, const at::Tensor& ws,
                  int64_t algo, double nu, const c10::optional<at::Tensor>& plan,
                  const c10::optional<at::Tensor>& plan_info) {
    check_coords(coords, "coords");
    const at::OptionalDeviceGuard guard(coords.device());
    check_nbr(nbr, coords);
    const int64_t rows = nbr.size(0), m = nbr.size(1), n = coords.size(0), d = coords.size(1);
    if (order.has_value()) {
        TORCH_CHECK(order->scalar_type() == at::kInt && order->sizes() == at::IntArrayRef{rows} && order->is_contiguous(),
                    "order must be a contiguous int32 (rows,) tensor");
        check_same_device(coords, *order, "order");
    }
    check_f64(values, {n}, coords, "values");
    check_f64(B, {rows, m}, coords, "B");
    check_f64(F, {rows}, coords, "F");
    check_f64(R, {rows}, coords, "R");
    check_f64(partials, {4}, coords, "partials");
    TORCH_CHECK(ws.is_contiguous(), "workspace must be contiguous");
    check_same_device(coords, ws, "workspace");
    if (plan.has_value()) {
        // a wave pair plan (pair_plan op): the pair kernel with every shared covariance evaluated once per wave
        TORCH_CHECK(plan_info.has_value() && plan_info->device().is_cpu() && plan_info->scalar_type() == at::kLong &&
                        plan_info->numel() == NNGP_PLAN_INFO_LEN && plan_info->is_contiguous(),
                    "plan_info must be the pair_plan op's CPU int64 (", NNGP_PLAN_INFO_LEN, ",) tensor");
        TORCH_CHECK(plan->scalar_type() == at::kByte && plan->is_contiguous(), "plan must be a contiguous uint8 tensor");
        check_same_device(coords, *plan, "plan");
        TORCH_CHECK(algo == NNGP_ALGO_AUTO || algo == NNGP_ALGO_PAIRB, "a pair plan runs the pair kernel (algo ", algo, ")");
        check_rc(nngp_bf_sweep_plan(coords.data_ptr<double>(), n, (int32_t)d, nbr.data_ptr<int32_t>(), ptr<int32_t>(order),
                                    rows, (int32_t)m, i0, (int32_t)kind, sigma2, phi, tau2, ptr<double>(values),
                                    ptr<double>(B), ptr<double>(F), ptr<double>(R), partials.data_ptr<double>(),
                                    ws.data_ptr(), (size_t)ws.nbytes(), plan->data_ptr(), (size_t)plan->nbytes(),
                                    plan_info->data_ptr<int64_t>(), stream(coords)),
                 "nngp_bf_sweep_plan");
        return;
    }
    check_rc(nngp_bf_sweep(coords.data_ptr<double>(), n, (int32_t)d, nbr.data_ptr<int32_t>(), ptr<int32_t>(order), rows,
                           (int32_t)m, i0, (int32_t)kind, sigma2, phi, tau2, nu, ptr<double>(values), ptr<double>(B),
                           ptr<double>(F), ptr<double>(R), partials.data_ptr<double>(), ws.data_ptr(),
                           (size_t)ws.nbytes(), (int32_t)algo, stream(coords)),
             "nngp_bf_sweep");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bf_sweep(const at::Tensor& coords, const at::Tensor& nbr, int64_t i0,
                                                        int64_t kind, double sigma2, double phi, double tau2,
                                                        const c10::optional<at::Tensor>& values, bool want_bf,
                                                        int64_t algo, const c10::optional<at::Tensor>& order,
                                                        double nu) {
    check_coords(coords, "coords");
    const at::OptionalDeviceGuard guard(coords.device());
    check_nbr(nbr, coords);
    const int64_t rows = nbr.size(0), m = nbr.size(1);
    auto f64 = coords.options();
    at::Tensor B = want_bf ? at::empty({rows, m}, f64) : at::empty({0, m}, f64);
    at::Tensor F = want_bf ? at::empty({rows}, f64) : at::empty({0}, f64);
    at::Tensor p = at::empty({4}, f64);
    auto ws = workspace((int64_t)nngp_bf_sweep_workspace_bytes(rows, (int32_t)m, (int32_t)kind,
                                                               (int32_t)coords.size(1), (int32_t)algo), coords);
    bf_sweep_out(coords, nbr, order, i0, kind, sigma2, phi, tau2, values,
                 want_bf ? c10::optional<at::Tensor>(B) : c10::nullopt,
                 want_bf ? c10::optional<at::Tensor>(F) : c10::nullopt, c10::nullopt, p, ws, algo, nu, c10::nullopt,
                 c10::nullopt);
    return {B, F, p};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bf_cross(const at::Tensor& ref, const at::Tensor& query,
                                                        const at::Tensor& nbr, int64_t kind, double sigma2, double phi,
                                                        double tau2, const c10::optional<at::Tensor>& ref_values,
                                                        int64_t algo, double nu) {
    check_coords(ref, "ref");
    const at::OptionalDeviceGuard guard(ref.device());
    check_coords(query, "query");
    check_same_device(ref, query, "query");
    TORCH_CHECK(ref.size(1) == query.size(1), "ref and query have different dimensions");
    check_nbr(nbr, ref);
    const int64_t rows = nbr.size(0), m = nbr.size(1), d = ref.size(1);
    check_f64(ref_values, {ref.size(0)}, ref, "ref_values");
    auto f64 = ref.options();
    at::Tensor B = at::empty({rows, m}, f64), F = at::empty({rows}, f64), R = at::empty({rows}, f64);
    at::Tensor p = at::empty({4}, f64);
    auto ws = workspace((int64_t)nngp_bf_sweep_workspace_bytes(rows, (int32_t)m, (int32_t)kind, (int32_t)d,
                                                               (int32_t)algo), ref);
    check_rc(nngp_bf_cross(ref.data_ptr<double>(), ref.size(0), (int32_t)d, query.data_ptr<double>(), query.size(0),
                           nbr.data_ptr<int32_t>(), nullptr, rows, (int32_t)m, 0, (int32_t)kind, sigma2, phi, tau2,
                           nu, ptr<double>(ref_values), nullptr, B.data_ptr<double>(), F.data_ptr<double>(),
                           ref_values.has_value() ? R.data_ptr<double>() : nullptr, p.data_ptr<double>(),
                           ws.data_ptr(), ws.nbytes(), (int32_t)algo, stream(ref)),
             "nngp_bf_cross");
    // R = 0 - B_t v_N: the kriging mean is -R (zeros without reference values)
    at::Tensor mean = ref_values.has_value() ? R.neg() : at::zeros({rows}, f64);
    return {B, F, mean};
}

// the wave pair plan of a sweep over nbr (include/nngp.h nngp_pair_plan_build): (plan bytes on the GPU,
// CPU int64 info).  A setup call: it synchronises the tensors' stream once.
std::tuple<at::Tensor, at::Tensor> pair_plan(const at::Tensor& nbr, const c10::optional<at::Tensor>& order, int64_t i0,
                                             int64_t n_points, int64_t dim) {
    TORCH_CHECK(nbr.is_cuda(), "nbr must be a ROCm GPU tensor (there is no CPU fallback)");
    const at::OptionalDeviceGuard guard(nbr.device());
    check_nbr(nbr, nbr);
    const int64_t rows = nbr.size(0), m = nbr.size(1);
    if (order.has_value()) {
        TORCH_CHECK(order->scalar_type() == at::kInt && order->sizes() == at::IntArrayRef{rows} && order->is_contiguous(),
                    "order must be a contiguous int32 (rows,) tensor");
        check_same_device(nbr, *order, "order");
    }
    const size_t bytes = nngp_pair_plan_bytes(rows, (int32_t)m, (int32_t)dim);
    TORCH_CHECK(bytes > 0, "no pair plans for m=", m, ", dim=", dim, " (2 <= m <= 17, dim 1..3)");
    auto plan = workspace((int64_t)bytes, nbr);
    auto info = at::empty({NNGP_PLAN_INFO_LEN}, at::TensorOptions().dtype(at::kLong));
    check_rc(nngp_pair_plan_build(nbr.data_ptr<int32_t>(), ptr<int32_t>(order), rows, (int32_t)m, i0, n_points,
                                  (int32_t)dim, plan.data_ptr(), (size_t)plan.nbytes(), info.data_ptr<int64_t>(),
                                  stream(nbr)),
             "nngp_pair_plan_build");
    return {plan, info};
}

std::tuple<at::Tensor, at::Tensor> row_order(const at::Tensor& coords, int64_t i0, int64_t rows,
                                             const c10::optional<at::Tensor>& nbr) {
    check_coords(coords, "coords");
    const at::OptionalDeviceGuard guard(coords.device());
    const int64_t n = coords.size(0);
    TORCH_CHECK(0 <= i0 && 0 <= rows && i0 + rows <= n, "rows [", i0, ", ", i0 + rows, ") outside [0, ", n, ")");
    int64_t m = 0;
    if (nbr.has_value()) {
        check_nbr(*nbr, coords);
        TORCH_CHECK(nbr->size(0) == rows, "nbr must have one row per location");
        m = nbr->size(1);
    }
    auto order = at::empty({rows}, coords.options().dtype(at::kInt));
    at::Tensor srt = nbr.has_value() ? at::empty_like(*nbr) : at::empty({0, 0}, coords.options().dtype(at::kInt));
    auto ws = workspace((int64_t)nngp_row_order_workspace_bytes(rows), coords);
    check_rc(nngp_row_order(coords.data_ptr<double>(), n, (int32_t)coords.size(1), ptr<int32_t>(nbr), (int32_t)m, i0,
                            rows, order.data_ptr<int32_t>(), nbr.has_value() ? srt.data_ptr<int32_t>() : nullptr,
                            ws.data_ptr(), ws.nbytes(), stream(coords)),
             "nngp_row_order");
    return {order, srt};
}

// gathered (world, 4) -> out (4,), or a batch of independent sweeps: gathered (world, n_slots, 4) -> out (n_slots, 4)
void combine_partials_out(const at::Tensor& gathered, const at::Tensor& out) {
    TORCH_CHECK(gathered.is_cuda() && gathered.scalar_type() == at::kDouble &&
                    (gathered.dim() == 2 || gathered.dim() == 3) && gathered.size(-1) == 4 && gathered.is_contiguous(),
                "gathered must be a contiguous float64 (world, 4) or (world, n_slots, 4) GPU tensor");
    const at::OptionalDeviceGuard guard(gathered.device());
    const int64_t slots = gathered.dim() == 3 ? gathered.size(1) : 1;
    if (gathered.dim() == 3)
        check_f64(out, {slots, 4}, gathered, "out");
    else
        check_f64(out, {4}, gathered, "out");
    check_rc(nngp_combine_partials_batch(gathered.data_ptr<double>(), (int32_t)gathered.size(0), slots,
                                         out.data_ptr<double>(), stream(gathered)),
             "nngp_combine_partials_batch");
}

}  // namespace

TORCH_LIBRARY(nngp, m) {
    m.def("knn_prior(Tensor coords, int m, int q0, int q1) -> Tensor");
    m.def("knn_prior_rows(Tensor coords, int m, Tensor rows) -> Tensor");
    m.def("knn_query(Tensor ref, Tensor query, int k) -> Tensor");
    m.def("bf_sweep(Tensor coords, Tensor nbr, int i0, int kind, float sigma2, float phi, float tau2, Tensor? values, "
          "bool want_bf, int algo, Tensor? order=None, float nu=-1.0) -> (Tensor, Tensor, Tensor)");
    m.def("bf_sweep_out(Tensor coords, Tensor nbr, Tensor? order, int i0, int kind, float sigma2, float phi, "
          "float tau2, Tensor? values, Tensor(a!)? B, Tensor(b!)? F, Tensor(c!)? R, Tensor(d!) partials, "
          "Tensor(e!) workspace, int algo, float nu=-1.0, Tensor? plan=None, Tensor? plan_info=None) -> ()");
    m.def("pair_plan(Tensor nbr, Tensor? order, int i0, int n_points, int dim) -> (Tensor, Tensor)");
    m.def("bf_cross(Tensor ref, Tensor query, Tensor nbr, int kind, float sigma2, float phi, float tau2, "
          "Tensor? ref_values, int algo, float nu=-1.0) -> (Tensor, Tensor, Tensor)");
    m.def("row_order(Tensor coords, int i0, int rows, Tensor? nbr) -> (Tensor, Tensor)");
    m.def("combine_partials_out(Tensor gathered, Tensor(a!) out) -> ()");
}

TORCH_LIBRARY_IMPL(nngp, CUDA, m) {
    m.impl("knn_prior", &knn_prior);
    m.impl("knn_prior_rows", &knn_prior_rows);
    m.impl("knn_query", &knn_query);
    m.impl("bf_sweep", &bf_sweep);
    m.impl("bf_sweep_out", &bf_sweep_out);
    m.impl("bf_cross", &bf_cross);
    m.impl("row_order", &row_order);
    m.impl("pair_plan", &pair_plan);
    m.impl("combine_partials_out", &combine_partials_out);
}
