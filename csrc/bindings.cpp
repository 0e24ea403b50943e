#include <cmath>
// Python bindings of the native runtime (module distributed_model_parallel_amd._C).
#include <torch/extension.h>
#include <torch/csrc/autograd/variable.h>

#include "comm/rccl_comm.h"
#include "ddp/reducer.h"
#include "dp/parallel_apply.h"

namespace dmp {
// batchnorm.hip
at::Tensor bn_local_moments(const at::Tensor& x, int64_t C);
std::vector<at::Tensor> bn_forward_apply(const at::Tensor& x, const at::Tensor& sums,
                                         const c10::optional<at::Tensor>& weight,
                                         const c10::optional<at::Tensor>& bias,
                                         const c10::optional<at::Tensor>& running_mean,
                                         const c10::optional<at::Tensor>& running_var,
                                         double momentum, double eps,
                                         const c10::optional<at::Tensor>& residual, bool relu,
                                         int64_t C,
                                         const c10::optional<at::Tensor>& num_batches_tracked,
                                         bool out_moments, double clip);
std::vector<at::Tensor> bn_eval_apply(const at::Tensor& x, const at::Tensor& running_mean,
                                      const at::Tensor& running_var,
                                      const c10::optional<at::Tensor>& weight,
                                      const c10::optional<at::Tensor>& bias, double eps,
                                      const c10::optional<at::Tensor>& residual, bool relu,
                                      int64_t C, double clip);
at::Tensor bn_backward_moments(const at::Tensor& dy, const at::Tensor& x,
                               const c10::optional<at::Tensor>& y, const at::Tensor& mean,
                               bool relu, int64_t C, const c10::optional<at::Tensor>& weight,
                               const c10::optional<at::Tensor>& bias,
                               const c10::optional<at::Tensor>& invstd, double clip);
at::Tensor bn_finalize(const at::Tensor& sums, const c10::optional<at::Tensor>& weight,
                       const c10::optional<at::Tensor>& bias,
                       const c10::optional<at::Tensor>& running_mean,
                       const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                       int64_t C, const c10::optional<at::Tensor>& num_batches_tracked);
std::vector<at::Tensor> bn_backward_apply(const at::Tensor& dy, const at::Tensor& x,
                                          const c10::optional<at::Tensor>& y,
                                          const at::Tensor& sums, const at::Tensor& count,
                                          const c10::optional<at::Tensor>& weight,
                                          const at::Tensor& mean, const at::Tensor& invstd,
                                          bool training, bool relu, bool want_dres, int64_t C,
                                          const c10::optional<at::Tensor>& bias, double clip,
                                          const c10::optional<at::Tensor>& acc_weight,
                                          const c10::optional<at::Tensor>& acc_bias);
// fused_sgd.hip
void sgd_flat_step(const c10::optional<at::Tensor>& master, const at::Tensor& mom,
                   const at::Tensor& grad, const at::Tensor& param, double lr, double wd,
                   double momentum, double dampening, bool nesterov, double grad_scale,
                   bool first_step);
// gemm_bf16.hip
std::vector<at::Tensor> gemm_nt(const at::Tensor& A, const at::Tensor& B,
                                const c10::optional<at::Tensor>& pro_scale,
                                const c10::optional<at::Tensor>& pro_shift, const std::string& mode,
                                const c10::optional<at::Tensor>& epi_scale,
                                const c10::optional<at::Tensor>& epi_shift,
                                const c10::optional<at::Tensor>& residual, bool relu,
                                const std::vector<int64_t>& a_map,
                                const std::vector<int64_t>& c_map,
                                const c10::optional<at::Tensor>& a2,
                                const std::vector<int64_t>& a2_map);
std::vector<at::Tensor> gemm_nt_bnbwd(const at::Tensor& A, const at::Tensor& B,
                                      const c10::optional<at::Tensor>& residual,
                                      const c10::optional<at::Tensor>& bn_x,
                                      const c10::optional<at::Tensor>& bn_y,
                                      const c10::optional<at::Tensor>& mean,
                                      const c10::optional<at::Tensor>& invstd,
                                      const c10::optional<at::Tensor>& weight,
                                      const c10::optional<at::Tensor>& bias,
                                      const std::vector<int64_t>& res_map,
                                      const c10::optional<at::Tensor>& a2,
                                      const c10::optional<at::Tensor>& ebias,
                                      const std::vector<int64_t>& a2_map);
// cross_entropy.hip
std::vector<at::Tensor> cross_entropy_fwd(const at::Tensor& x, const at::Tensor& target,
                                          int64_t ignore_index, double scale,
                                          const c10::optional<at::Tensor>& acc);
at::Tensor cross_entropy_bwd(const at::Tensor& grad, const at::Tensor& x, const at::Tensor& target,
                             const at::Tensor& lse, const at::Tensor& stats, int64_t ignore_index);
at::Tensor gemm_tn(const at::Tensor& A, const at::Tensor& B, at::ScalarType out_dtype,
                   const std::vector<int64_t>& b_map, const c10::optional<at::Tensor>& pro_scale,
                   const c10::optional<at::Tensor>& pro_shift, bool a_mapped,
                   const c10::optional<at::Tensor>& out);
// stem.hip
at::Tensor space_to_depth2(const at::Tensor& x, int64_t pad, int64_t out_channels);
at::Tensor pad_channels16(const at::Tensor& x, int64_t pad, int64_t extra_w);
// maxpool.hip (fused stem BN + pool)
std::vector<at::Tensor> maxpool2d_bn_forward(const at::Tensor& x, const at::Tensor& scale,
                                             const at::Tensor& shift, int64_t k, int64_t s, int64_t p);
std::vector<at::Tensor> maxpool2d_bn_backward(const at::Tensor& dy, const at::Tensor& idx, const at::Tensor& x,
                                              const at::Tensor& scale, const at::Tensor& shift,
                                              const at::Tensor& mean, int64_t k, int64_t s, int64_t p);
std::vector<at::Tensor> conv_nt(const at::Tensor& x, const at::Tensor& wmat, int64_t kh,
                                int64_t kw, int64_t stride, int64_t pad, int64_t ho, int64_t wo,
                                bool transposed, const c10::optional<at::Tensor>& pro_scale,
                                const c10::optional<at::Tensor>& pro_shift,
                                const std::string& mode,
                                const c10::optional<at::Tensor>& epi_scale,
                                const c10::optional<at::Tensor>& epi_shift,
                                const c10::optional<at::Tensor>& residual, bool relu,
                                int64_t kc);
void set_gemm_tile(int64_t t);
void set_phase_dgrad(bool on);
void set_tn_wide(bool on);
at::Tensor conv_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t kh, int64_t kw,
                      int64_t stride, int64_t pad, int64_t ho, int64_t wo,
                      at::ScalarType out_dtype, int64_t kc, const c10::optional<at::Tensor>& out);
// gemm_xl.hip
at::Tensor gemm_xl(const at::Tensor& A, const at::Tensor& B, const std::string& mode,
                   const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& aux,
                   const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& out);
void set_gemm_xl_bn(int bn, int pipe, int group_m);
int get_gemm_xl_pipe();
void set_gemm_xl_x2(int mode);
int get_gemm_xl_x2();
void set_gemm_xl_bm(int bm);
void set_gemm_xl_trace(const c10::optional<at::Tensor>& buf);
int get_gemm_xl_bm(int64_t M, int64_t N, int64_t K);
std::vector<at::Tensor> conv_xl(const at::Tensor& x, const at::Tensor& wmat, int64_t kh, int64_t kw,
                                int64_t stride, int64_t pad, int64_t ho, int64_t wo, const std::string& mode,
                                const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& bn_x,
                                const c10::optional<at::Tensor>& bn_y, const c10::optional<at::Tensor>& mean,
                                const c10::optional<at::Tensor>& invstd, const c10::optional<at::Tensor>& weight,
                                const c10::optional<at::Tensor>& bias);
std::vector<at::Tensor> gemm_xl_dgelu_bgrad(const at::Tensor& A, const at::Tensor& B, const at::Tensor& aux);
at::Tensor gemm_tn_xl(const at::Tensor& A, const at::Tensor& B, at::ScalarType out_dtype,
                      const c10::optional<at::Tensor>& out);
at::Tensor gram_strided_xl(const at::Tensor& x, int64_t stride, int64_t ho, int64_t wo);
bool gram_strided_xl_supported(int64_t nb, int64_t cin, int64_t hi, int64_t wi, int64_t ho, int64_t wo);
// conv3x3_halo.hip
std::vector<at::Tensor> conv3x3_c64(const at::Tensor& x, const at::Tensor& wmat, bool moments);
std::vector<at::Tensor> conv3x3_c128(const at::Tensor& x, const at::Tensor& wmat, bool moments);
bool conv3x3_c128_supported(int64_t c, int64_t h, int64_t w);
at::Tensor conv3x3_c128_dgrad_s2(const at::Tensor& dy, const at::Tensor& wt);
void set_bn_streaming(bool on);
at::Tensor conv_xl_dgrad_s2(const at::Tensor& dy, const std::vector<at::Tensor>& wph, int64_t hi, int64_t wi);
void set_pool_generic(bool on);
at::Tensor wgrad3x3(const at::Tensor& dy, const at::Tensor& x, int64_t stride);
bool stem_halo_supported(int64_t hs, int64_t ws, int64_t ho, int64_t wo);
std::vector<at::Tensor> stem_halo_fwd(const at::Tensor& s, const at::Tensor& wm, int64_t ho, bool moments);
at::Tensor stem_halo_wgrad(const at::Tensor& dy, const at::Tensor& s, int64_t ho, at::ScalarType out_dtype);
at::Tensor stem_fold_finish(const at::Tensor& img, int64_t ho, int64_t wo, const at::Tensor& t_dz,
                            const at::Tensor& t_y, const at::Tensor& sums, const at::Tensor& cnt,
                            const at::Tensor& invstd, const c10::optional<at::Tensor>& weight, const at::Tensor& mean,
                            at::ScalarType out_dtype);
bool wgrad3x3_supported(int64_t C, int64_t H, int64_t W, int64_t stride);
void set_wgrad3x3_waves(int64_t nw);
void set_tn_xl_rounds(int r);
void set_tn_narrow(bool on);
void set_gemm_xl_trim_heavy(bool on);
at::Tensor conv_wgrad_xl(const at::Tensor& dy, const at::Tensor& x, int64_t kh, int64_t kw, int64_t stride,
                         int64_t pad, int64_t ho, int64_t wo, at::ScalarType out_dtype,
                         const c10::optional<at::Tensor>& out);
std::vector<at::Tensor> gemm_xl_conv(const at::Tensor& A, const at::Tensor& B, const std::string& mode,
                                     const c10::optional<at::Tensor>& residual,
                                     const c10::optional<at::Tensor>& bn_x,
                                     const c10::optional<at::Tensor>& bn_y,
                                     const c10::optional<at::Tensor>& mean,
                                     const c10::optional<at::Tensor>& invstd,
                                     const c10::optional<at::Tensor>& weight,
                                     const c10::optional<at::Tensor>& bias,
                                     const std::vector<int64_t>& res_map,
                                     const c10::optional<at::Tensor>& a2,
                                     const c10::optional<at::Tensor>& ebias,
                                     const c10::optional<at::Tensor>& scale,
                                     const c10::optional<at::Tensor>& shift, bool relu,
                                     const std::vector<int64_t>& a2_map);
// bn_fold.hip
bool bn_fold_supported(int64_t cout, int64_t cin);
std::vector<at::Tensor> bn_fold_fwd(const at::Tensor& W, const at::Tensor& G, const at::Tensor& asums,
                                    const c10::optional<at::Tensor>& Wf);
std::vector<at::Tensor> bn_fold_fwd_finalize(const at::Tensor& W, const at::Tensor& G, const at::Tensor& asums,
                                             const c10::optional<at::Tensor>& Wf,
                                             const c10::optional<at::Tensor>& weight,
                                             const c10::optional<at::Tensor>& bias,
                                             const c10::optional<at::Tensor>& running_mean,
                                             const c10::optional<at::Tensor>& running_var, double momentum,
                                             double eps, const c10::optional<at::Tensor>& num_batches_tracked);
at::Tensor bn_fold_bwd_sums(const at::Tensor& D, const at::Tensor& W, const at::Tensor& sdz,
                            const at::Tensor& mean);
std::vector<at::Tensor> bn_fold_bwd_coef(const at::Tensor& sums, const at::Tensor& local, const at::Tensor& count,
                                         const at::Tensor& invstd, const at::Tensor& mean,
                                         const c10::optional<at::Tensor>& gamma, const at::Tensor& D,
                                         const at::Tensor& WG, const at::Tensor& s, const at::Tensor& W);
std::vector<at::Tensor> bn_fold_relu_mask(const at::Tensor& dy, const at::Tensor& y);
at::Tensor bn_fold_colsum(const at::Tensor& x, const std::vector<int64_t>& map);
std::vector<at::Tensor> bn_fold_scale_concat(const at::Tensor& W3, const at::Tensor& s3, const at::Tensor& t3,
                                             const at::Tensor& Wd, const at::Tensor& sd, const at::Tensor& td);
// attention.hip
bool attention_supported(int64_t S, int64_t head_dim);
void set_attention_variant(int fwd, int bwd);
void set_fold_gemm(int mode);
int get_fold_gemm();
std::vector<int64_t> get_attention_variant();
std::vector<at::Tensor> attention_forward(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, double scale);
at::Tensor attention_backward(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o,
                              const at::Tensor& lse, int64_t B, int64_t S, int64_t H, double scale);
// depthwise.hip
std::vector<at::Tensor> dwconv3x3_forward(const at::Tensor& x, const at::Tensor& w, int64_t stride,
                                          bool moments);
at::Tensor dwconv3x3_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t stride, int64_t H,
                           int64_t W);
at::Tensor dwconv3x3_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t stride,
                           at::ScalarType out_dtype, const c10::optional<at::Tensor>& out);
// bias_act.hip
bool colsum_supported(int64_t N);
at::Tensor bias_grad(const at::Tensor& dy, at::ScalarType out_dtype);
std::vector<at::Tensor> gelu_bwd_bias_grad(const at::Tensor& dy, const at::Tensor& h, at::ScalarType out_dtype);
// layernorm.hip
std::vector<at::Tensor> layernorm_forward(const at::Tensor& x, const c10::optional<at::Tensor>& w,
                                          const c10::optional<at::Tensor>& b, int64_t D,
                                          double eps);
std::vector<at::Tensor> layernorm_backward(const at::Tensor& dy, const at::Tensor& x,
                                           const c10::optional<at::Tensor>& w,
                                           const at::Tensor& mean, const at::Tensor& rstd,
                                           int64_t D, at::ScalarType param_dtype,
                                           const c10::optional<at::Tensor>& dres);
bool layernorm_supported(int64_t D);
// maxpool.hip
std::vector<at::Tensor> maxpool2d_forward(const at::Tensor& x, int64_t k, int64_t s, int64_t p);
at::Tensor global_avgpool_backward(const at::Tensor& g, int64_t H, int64_t W);
at::Tensor maxpool2d_backward(const at::Tensor& dy, const at::Tensor& idx, int64_t H, int64_t W,
                              int64_t k, int64_t s, int64_t p);
// coalesced.hip
void multi_copy(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts);
void multi_transpose(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
                     const std::vector<int64_t>& taps);
void multi_cast_bf16_f32(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts);
void reduce_add_into(const std::vector<at::Tensor>& inputs, at::Tensor& out);
void gather_slabs(const std::vector<at::Tensor>& inputs, at::Tensor& out, bool along_inner);
std::vector<std::vector<bool>> enable_peer_access(int64_t num_devices);
}  // namespace dmp

namespace py = pybind11;

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native runtime: RCCL communicator, DDP reducer, HIP kernels (gfx950)";

  // ---- batch norm ----
  m.def("bn_local_moments", &dmp::bn_local_moments,
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_forward_apply", &dmp::bn_forward_apply, py::arg("x"), py::arg("sums"), py::arg("weight"),
        py::arg("bias"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"),
        py::arg("eps"), py::arg("residual"), py::arg("relu"), py::arg("C"),
        py::arg("num_batches_tracked") = py::none(), py::arg("out_moments") = false,
        py::arg("clip") = INFINITY,
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_eval_apply", &dmp::bn_eval_apply, py::arg("x"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("weight"), py::arg("bias"), py::arg("eps"), py::arg("residual"),
        py::arg("relu"), py::arg("C"), py::arg("clip") = INFINITY,
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_finalize", &dmp::bn_finalize, py::arg("sums"), py::arg("weight"), py::arg("bias"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("C"), py::arg("num_batches_tracked") = py::none(),
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_backward_moments", &dmp::bn_backward_moments, py::arg("dy"), py::arg("x"), py::arg("y"),
        py::arg("mean"), py::arg("relu"), py::arg("C"), py::arg("weight") = py::none(),
        py::arg("bias") = py::none(), py::arg("invstd") = py::none(), py::arg("clip") = INFINITY,
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_backward_apply", &dmp::bn_backward_apply, py::arg("dy"), py::arg("x"), py::arg("y"),
        py::arg("sums"), py::arg("count"), py::arg("weight"), py::arg("mean"), py::arg("invstd"),
        py::arg("training"), py::arg("relu"), py::arg("want_dres"), py::arg("C"),
        py::arg("bias") = py::none(), py::arg("clip") = INFINITY, py::arg("acc_weight") = py::none(),
        py::arg("acc_bias") = py::none(),
        py::call_guard<py::gil_scoped_release>());

  // ---- MFMA GEMM (1x1 conv) with fused BN prologue/epilogues ----
  m.def("gemm_nt", &dmp::gemm_nt, py::arg("A"), py::arg("B"), py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("mode") = "store",
        py::arg("epi_scale") = py::none(), py::arg("epi_shift") = py::none(),
        py::arg("residual") = py::none(), py::arg("relu") = false,
        py::arg("a_map") = std::vector<int64_t>{}, py::arg("c_map") = std::vector<int64_t>{},
        py::arg("a2") = py::none(), py::arg("a2_map") = std::vector<int64_t>{},
        py::call_guard<py::gil_scoped_release>());

  m.def("cross_entropy_fwd", &dmp::cross_entropy_fwd, py::arg("x"), py::arg("target"),
        py::arg("ignore_index") = -100, py::arg("scale") = 1.0, py::arg("acc") = py::none(),
        "scale * mean softmax cross-entropy; acc (fp64 [3]) += (loss, top-1 correct, top-5 correct)",
        py::call_guard<py::gil_scoped_release>());
  m.def("cross_entropy_bwd", &dmp::cross_entropy_bwd, py::arg("grad"), py::arg("x"), py::arg("target"),
        py::arg("lse"), py::arg("stats"), py::arg("ignore_index") = -100,
        py::call_guard<py::gil_scoped_release>());
  m.def("gemm_nt_bnbwd", &dmp::gemm_nt_bnbwd, py::arg("A"), py::arg("B"), py::arg("residual"),
        py::arg("bn_x"), py::arg("bn_y"), py::arg("mean"), py::arg("invstd"), py::arg("weight"),
        py::arg("bias"), py::arg("res_map") = std::vector<int64_t>{}, py::arg("a2") = py::none(),
        py::arg("ebias") = py::none(), py::arg("a2_map") = std::vector<int64_t>{},
        py::call_guard<py::gil_scoped_release>());

  m.def("gemm_tn", &dmp::gemm_tn, py::arg("A"), py::arg("B"), py::arg("out_dtype"),
        py::arg("b_map") = std::vector<int64_t>{}, py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("a_mapped") = false, py::arg("out") = py::none(),
        "C = A^T B (weight gradient); b_map reads B's rows through a strided map, a_mapped A's too (Gram of a "
        "sample); out: add into this gradient instead of returning a new tensor",
        py::call_guard<py::gil_scoped_release>());

  m.def("set_tn_wide", &dmp::set_tn_wide, py::arg("on"),
        "128 x 256 TN tiles for deep weight gradients (default on)");
  m.def("set_phase_dgrad", &dmp::set_phase_dgrad, py::arg("on"),
        "strided implicit-GEMM data gradients as stride-phase launches (default on)");
  m.def("set_gemm_tile", &dmp::set_gemm_tile,
        "debug: force the NT GEMM tile variant (-1 auto, 0 256x64, 1 128x64, 2 128x128, "
        "3 128x64/4x1, 4 64x128, 5 64x64)");

  // ---- implicit-GEMM convolution (kh x kw taps) on the same MFMA kernels ----
  m.def("conv_nt", &dmp::conv_nt, py::arg("x"), py::arg("wmat"), py::arg("kh"), py::arg("kw"),
        py::arg("stride"), py::arg("pad"), py::arg("ho"), py::arg("wo"),
        py::arg("transposed") = false, py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("mode") = "store",
        py::arg("epi_scale") = py::none(), py::arg("epi_shift") = py::none(),
        py::arg("residual") = py::none(), py::arg("relu") = false, py::arg("kc") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("conv_wgrad", &dmp::conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("kh"), py::arg("kw"),
        py::arg("stride"), py::arg("pad"), py::arg("ho"), py::arg("wo"), py::arg("out_dtype"),
        py::arg("kc") = 0, py::arg("out") = py::none(),
        py::call_guard<py::gil_scoped_release>());
  m.def("maxpool2d_bn_forward", &dmp::maxpool2d_bn_forward, py::arg("x"), py::arg("scale"),
        py::arg("shift"), py::arg("k"), py::arg("s"), py::arg("p"),
        py::call_guard<py::gil_scoped_release>());
  m.def("maxpool2d_bn_backward", &dmp::maxpool2d_bn_backward, py::arg("dy"), py::arg("idx"), py::arg("x"),
        py::arg("scale"), py::arg("shift"), py::arg("mean"), py::arg("k"), py::arg("s"), py::arg("p"),
        py::call_guard<py::gil_scoped_release>());
  m.def("pad_channels16", &dmp::pad_channels16, py::arg("x"), py::arg("pad"), py::arg("extra_w") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("space_to_depth2", &dmp::space_to_depth2, py::arg("x"), py::arg("pad"), py::arg("out_channels") = 16,
        py::call_guard<py::gil_scoped_release>());

  // ---- large-tile transformer GEMM with fused bias / GELU / residual epilogues ----
  m.def("gemm_xl", &dmp::gemm_xl, py::arg("A"), py::arg("B"), py::arg("mode") = "store",
        py::arg("bias") = py::none(), py::arg("aux") = py::none(),
        py::arg("residual") = py::none(), py::arg("out") = py::none(),
        py::call_guard<py::gil_scoped_release>());
  m.def("conv_xl", &dmp::conv_xl, py::arg("x"), py::arg("wmat"), py::arg("kh"), py::arg("kw"),
        py::arg("stride"), py::arg("pad"), py::arg("ho"), py::arg("wo"), py::arg("mode") = "moments",
        py::arg("residual") = py::none(), py::arg("bn_x") = py::none(), py::arg("bn_y") = py::none(),
        py::arg("mean") = py::none(), py::arg("invstd") = py::none(), py::arg("weight") = py::none(),
        py::arg("bias") = py::none(),
        "Implicit-GEMM conv (NHWC gather) on the 256x256 ping-pong MFMA kernel with conv epilogues",
        py::call_guard<py::gil_scoped_release>());
  m.def("stem_halo_supported", &dmp::stem_halo_supported);
  m.def("stem_halo_fwd", &dmp::stem_halo_fwd, py::arg("s"), py::arg("wm"), py::arg("ho"), py::arg("moments") = false,
        "ResNet stem (s2d 4x4 conv, 16 -> 64 ch, Wo = 112) forward: halo-tiled, weights in VGPRs",
        py::call_guard<py::gil_scoped_release>());
  m.def("stem_fold_finish", &dmp::stem_fold_finish, py::arg("img"), py::arg("ho"), py::arg("wo"), py::arg("t_dz"),
        py::arg("t_y"), py::arg("sums"), py::arg("cnt"), py::arg("invstd"), py::arg("weight"), py::arg("mean"),
        py::arg("out_dtype"),
        "folded stem weight gradient: BN-backward coefficients, the 16 window sums of the batch-summed "
        "space-to-depth image, and al t_dz + be t_y + cc cols in one launch",
        py::call_guard<py::gil_scoped_release>());
  m.def("stem_halo_wgrad", &dmp::stem_halo_wgrad, py::arg("dy"), py::arg("s"), py::arg("ho"), py::arg("out_dtype"),
        "ResNet stem weight gradient [64, 256]: halo-tiled, dW in VGPRs",
        py::call_guard<py::gil_scoped_release>());
  m.def("wgrad3x3", &dmp::wgrad3x3, py::arg("dy"), py::arg("x"), py::arg("stride") = 1,
        "dW [C, C, 3, 3] (channels_last) of a 3x3/s1/p1 conv: persistent halo-tiled MFMA kernel",
        py::call_guard<py::gil_scoped_release>());
  m.def("wgrad3x3_supported", &dmp::wgrad3x3_supported, py::arg("C"), py::arg("Ho"), py::arg("Wo"),
        py::arg("stride") = 1);
  m.def("set_wgrad3x3_waves", &dmp::set_wgrad3x3_waves);
  m.def("conv3x3_c64", &dmp::conv3x3_c64, py::arg("x"), py::arg("wmat"), py::arg("moments") = false,
        "3x3/s1/p1 64->64-channel conv (W = 56) on the persistent halo-tiled MFMA kernel; "
        "returns (y [N*H*W, 64], fp64 moments [129] or empty)",
        py::call_guard<py::gil_scoped_release>());
  m.def("conv3x3_c128", &dmp::conv3x3_c128, py::arg("x"), py::arg("wmat"), py::arg("moments") = false,
        "3x3/s1/p1 128->128-channel conv (W = 28, H % 4 == 0) on the persistent halo-tiled MFMA kernel "
        "(Cout split over grid halves, K split over wave pairs); returns (y [N*H*W, 128], fp64 moments [257] or empty)",
        py::call_guard<py::gil_scoped_release>());
  m.def("conv3x3_c128_dgrad_s2", &dmp::conv3x3_c128_dgrad_s2, py::arg("dy"), py::arg("wt"),
        "data gradient of a 3x3/s2/p1 128->128 conv (dy 28 wide) as its four stride phases on the halo kernel; "
        "wt = W.permute(1, 2, 3, 0) as [128, 1152]; returns dx [N*2H*56, 128]",
        py::call_guard<py::gil_scoped_release>());
  m.def("conv3x3_c128_supported", &dmp::conv3x3_c128_supported, py::arg("C"), py::arg("H"), py::arg("W"));
  m.def("conv_xl_dgrad_s2", &dmp::conv_xl_dgrad_s2, py::arg("dy"), py::arg("wph"), py::arg("hi"), py::arg("wi"),
        "data gradient of a 3x3/s2/p1 conv as four stride-phase implicit GEMMs on the ping-pong kernel; "
        "returns dx [N*hi*wi, Cin]",
        py::call_guard<py::gil_scoped_release>());
  m.def("set_bn_streaming", &dmp::set_bn_streaming, py::arg("on"),
        "A/B: non-temporal streaming in the BN apply passes over > 256 MB tensors (default on)");
  m.def("set_pool_generic", &dmp::set_pool_generic, py::arg("on"),
        "A/B: route every max-pool geometry through the runtime-k kernels (default off)");
  m.def("set_tn_xl_rounds", &dmp::set_tn_xl_rounds, py::arg("rounds"));
  m.def("set_gemm_xl_trim_heavy", &dmp::set_gemm_xl_trim_heavy, py::arg("on"),
        "A/B: trimmed (192..240-row) tiles for the PIPE-10 heavy-epilogue GEMMs at any K (default on)");
  m.def("set_tn_narrow", &dmp::set_tn_narrow, py::arg("on"),
        "A/B: 4-wave weight-gradient tiles of 64 / 128 on an output side that narrow (default on)");
  m.def("gemm_tn_xl", &dmp::gemm_tn_xl, py::arg("A"), py::arg("B"), py::arg("out_dtype"), py::arg("out") = py::none(),
        "A^T B (weight gradient) on the ping-pong MFMA schedule, split over M",
        py::call_guard<py::gil_scoped_release>());
  m.def("gram_strided_xl", &dmp::gram_strided_xl, py::arg("x"), py::arg("stride"), py::arg("ho"), py::arg("wo"),
        "fp32 Gram x_s^T x_s of the stride-s sample of an NHWC bf16 input (4-wave TN kernel, both operands gathered)",
        py::call_guard<py::gil_scoped_release>());
  m.def("gram_strided_xl_supported", &dmp::gram_strided_xl_supported);
  m.def("conv_wgrad_xl", &dmp::conv_wgrad_xl, py::arg("dy"), py::arg("x"), py::arg("kh"), py::arg("kw"),
        py::arg("stride"), py::arg("pad"), py::arg("ho"), py::arg("wo"), py::arg("out_dtype"),
        py::arg("out") = py::none(),
        "kh x kw conv weight gradient (tap gather) on the ping-pong TN kernel; Cin % 256 == 0",
        py::call_guard<py::gil_scoped_release>());
  m.def("gemm_xl_dgelu_bgrad", &dmp::gemm_xl_dgelu_bgrad, py::arg("A"), py::arg("B"), py::arg("aux"),
        py::call_guard<py::gil_scoped_release>());
  m.def("gemm_xl_conv", &dmp::gemm_xl_conv, py::arg("A"), py::arg("B"), py::arg("mode"),
        py::arg("residual") = py::none(), py::arg("bn_x") = py::none(), py::arg("bn_y") = py::none(),
        py::arg("mean") = py::none(), py::arg("invstd") = py::none(), py::arg("weight") = py::none(),
        py::arg("bias") = py::none(), py::arg("res_map") = std::vector<int64_t>{},
        py::arg("a2") = py::none(), py::arg("ebias") = py::none(), py::arg("scale") = py::none(),
        py::arg("shift") = py::none(), py::arg("relu") = false, py::arg("a2_map") = std::vector<int64_t>{},
        "wide 1x1-conv GEMM with conv epilogues: moments | add | bnbwd | affine (scale, shift, residual, relu); "
        "a2: second A source concatenated along K; ebias: bnbwd per-column constant",
        py::call_guard<py::gil_scoped_release>());
  m.def("get_gemm_xl_pipe", &dmp::get_gemm_xl_pipe);
  m.def("set_gemm_xl_x2", &dmp::set_gemm_xl_x2, py::arg("mode"),
        "conv-epilogue GEMMs on the two-blocks-per-CU 256x128 kernel: 0 off, 1 where N % 256 != 0, 2 always");
  m.def("get_gemm_xl_x2", &dmp::get_gemm_xl_x2);
  m.def("set_gemm_xl_bm", &dmp::set_gemm_xl_bm, py::arg("bm"),
        "256x256 ping-pong GEMMs: rows per tile (0 auto: trimmed to fill whole rounds when K >= 768; "
        "-1 always 256; 192..240 forced)");
  m.def("set_gemm_xl_trace", &dmp::set_gemm_xl_trace, py::arg("buf") = py::none(),
        "diagnostics: 256x256 ping-pong GEMM launches record per-block phase timestamps into buf "
        "(int64 [blocks * 8]: entry, operands landed, main loop done, epilogue done, HW_ID, XCC_ID); None = off");
  m.def("get_gemm_xl_bm", &dmp::get_gemm_xl_bm, py::arg("M"), py::arg("N"), py::arg("K"),
        "rows per tile the ping-pong GEMM would take for this shape");
  m.def("set_gemm_xl_bn", &dmp::set_gemm_xl_bn, py::arg("bn"), py::arg("pipe") = -1, py::arg("group_m") = 0,
        "debug: force the gemm_xl N tile (0 auto, 128, 256) and main loop (0, 1, 10, 11; -1 default)");

  // ---- BN folded through an expanding 1x1 conv (ops/bn_fold.py) ----
  m.def("bn_fold_supported", &dmp::bn_fold_supported, py::arg("cout"), py::arg("cin"));
  m.def("bn_fold_fwd_finalize", &dmp::bn_fold_fwd_finalize, py::arg("W"), py::arg("G"), py::arg("asums"),
        py::arg("Wf"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"), py::arg("running_var"),
        py::arg("momentum"), py::arg("eps"), py::arg("num_batches_tracked"),
        "bn_fold_fwd + the BN finalize of its moments in one launch: (sums, WG, coef[4, Cout])");
  m.def("bn_fold_fwd", &dmp::bn_fold_fwd, py::arg("W"), py::arg("G"), py::arg("asums"), py::arg("Wf") = py::none(),
        "(sums fp64 [2Cout+1], WG fp32 [Cout, Cin]) of y = a W^T from G = a^T a and colsum(a)",
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_fold_bwd_sums", &dmp::bn_fold_bwd_sums, py::arg("D"), py::arg("W"), py::arg("sdz"), py::arg("mean"),
        "local fp64 [2Cout] = (sum dz, sum dz*(y - mean)) from D = dz^T a",
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_fold_bwd_coef", &dmp::bn_fold_bwd_coef, py::arg("sums"), py::arg("local"), py::arg("count"),
        py::arg("invstd"), py::arg("mean"), py::arg("gamma"), py::arg("D"), py::arg("WG"), py::arg("s"),
        py::arg("W"), "(dW, dgamma, dbeta, Bm = [(al o W)^T | W^T diag(be) W], ebias = c^T W)",
        py::call_guard<py::gil_scoped_release>());

  m.def("bn_fold_relu_mask", &dmp::bn_fold_relu_mask, py::arg("dy"), py::arg("y"),
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_fold_colsum", &dmp::bn_fold_colsum, py::arg("x"), py::arg("map") = std::vector<int64_t>{},
        "fp64 [2C+1] (colsum, colsum of squares, rows) of x's rows sampled through a strided map",
        py::call_guard<py::gil_scoped_release>());
  m.def("bn_fold_scale_concat", &dmp::bn_fold_scale_concat, py::arg("W3"), py::arg("s3"), py::arg("t3"),
        py::arg("Wd"), py::arg("sd"), py::arg("td"), "([s3 o W3 | sd o Wd] bf16, t3 + td)",
        py::call_guard<py::gil_scoped_release>());

  // ---- fused self-attention on packed qkv (ViT) ----
  m.def("attention_supported", &dmp::attention_supported);
  m.def("set_fold_gemm", &dmp::set_fold_gemm, py::arg("mode"),
        "BN-fold coefficient products: 0 fused VALU kernels, 1 library fp32 GEMMs (default), 2 tiled kernel");
  m.def("get_fold_gemm", &dmp::get_fold_gemm);
  m.def("get_attention_variant", &dmp::get_attention_variant);
  m.def("set_attention_variant", &dmp::set_attention_variant, py::arg("fwd"), py::arg("bwd") = 1,
        "attention kernels: fwd 0 = one workgroup per (batch, head), 1 = persistent with next-head prefetch, "
        "2 = 8-wave per head; bwd 0 = per head, 1 = persistent with prefetch");
  m.def("attention_forward", &dmp::attention_forward, py::arg("qkv"), py::arg("B"), py::arg("S"),
        py::arg("H"), py::arg("scale"),
        py::call_guard<py::gil_scoped_release>());
  m.def("attention_backward", &dmp::attention_backward, py::arg("dout"), py::arg("qkv"), py::arg("o"),
        py::arg("lse"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("scale"),
        py::call_guard<py::gil_scoped_release>());

  // ---- Linear side passes: bias gradient, GELU backward + bias gradient ----
  m.def("colsum_supported", &dmp::colsum_supported);
  m.def("bias_grad", &dmp::bias_grad, py::arg("dy"), py::arg("out_dtype"),
        py::call_guard<py::gil_scoped_release>());
  m.def("gelu_bwd_bias_grad", &dmp::gelu_bwd_bias_grad, py::arg("dy"), py::arg("h"), py::arg("out_dtype"),
        py::call_guard<py::gil_scoped_release>());

  // ---- LayerNorm (last dim) ----
  m.def("layernorm_forward", &dmp::layernorm_forward,
        py::call_guard<py::gil_scoped_release>());
  m.def("layernorm_backward", &dmp::layernorm_backward, py::arg("dy"), py::arg("x"), py::arg("w"),
        py::arg("mean"), py::arg("rstd"), py::arg("D"), py::arg("param_dtype"),
        py::arg("dres") = py::none(),
        py::call_guard<py::gil_scoped_release>());
  m.def("layernorm_supported", &dmp::layernorm_supported);

  // ---- NHWC max pooling with byte argmax ----
  m.def("maxpool2d_forward", &dmp::maxpool2d_forward,
        py::call_guard<py::gil_scoped_release>());
  m.def("maxpool2d_backward", &dmp::maxpool2d_backward,
        py::call_guard<py::gil_scoped_release>());
  m.def("global_avgpool_backward", &dmp::global_avgpool_backward,
        py::call_guard<py::gil_scoped_release>());

  // ---- depthwise 3x3 (NHWC) ----
  m.def("dwconv3x3_forward", &dmp::dwconv3x3_forward, py::arg("x"), py::arg("w"),
        py::arg("stride"), py::arg("moments") = false,
        py::call_guard<py::gil_scoped_release>());
  m.def("dwconv3x3_dgrad", &dmp::dwconv3x3_dgrad,
        py::call_guard<py::gil_scoped_release>());
  m.def("dwconv3x3_wgrad", &dmp::dwconv3x3_wgrad, py::arg("dy"), py::arg("x"), py::arg("stride"),
        py::arg("out_dtype"), py::arg("out") = py::none(),
        py::call_guard<py::gil_scoped_release>());

  // ---- optimizer ----
  m.def("sgd_flat_step", &dmp::sgd_flat_step,
        py::call_guard<py::gil_scoped_release>());

  // ---- coalesced movement ----
  m.def("multi_copy", &dmp::multi_copy,
        py::call_guard<py::gil_scoped_release>());
  m.def("multi_cast_bf16_f32", &dmp::multi_cast_bf16_f32, py::arg("srcs"), py::arg("dsts"),
        "dst[i] (fp32) = src[i] (bf16) for contiguous tensors, up to 64 per launch",
        py::call_guard<py::gil_scoped_release>());
  m.def("multi_transpose", &dmp::multi_transpose, py::arg("srcs"), py::arg("dsts"),
        py::arg("taps") = std::vector<int64_t>{},
        "dst[i] = src[i]^T for contiguous 2-byte matrices, up to 64 per launch; taps[i] = T (-T: "
        "flipped) transposes [R, T*C] -> [C, T*R] tap by tap",
        py::call_guard<py::gil_scoped_release>());
  m.def("reduce_add_into", &dmp::reduce_add_into,
        py::call_guard<py::gil_scoped_release>());
  m.def("gather_slabs", &dmp::gather_slabs,
        py::call_guard<py::gil_scoped_release>());
  m.def("enable_peer_access", &dmp::enable_peer_access);

  // ---- RCCL ----
  py::class_<dmp::RcclComm, std::shared_ptr<dmp::RcclComm>>(m, "RcclComm")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, bool>(), py::arg("unique_id"),
           py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("high_priority") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("set_inline", &dmp::RcclComm::set_inline)
      .def("is_inline", &dmp::RcclComm::is_inline)
      .def_static("new_unique_id", [] { return py::bytes(dmp::RcclComm::new_unique_id()); })
      .def_property_readonly("rank", &dmp::RcclComm::rank)
      .def_property_readonly("size", &dmp::RcclComm::size)
      .def_property_readonly("device", &dmp::RcclComm::device)
      .def("all_reduce", &dmp::RcclComm::all_reduce, py::arg("tensor"), py::arg("op") = "sum",
           py::arg("on_current_stream") = false, py::call_guard<py::gil_scoped_release>())
      .def("all_reduce_coalesced", &dmp::RcclComm::all_reduce_coalesced, py::arg("tensors"),
           py::arg("op") = "sum", py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &dmp::RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("reduce", &dmp::RcclComm::reduce, py::arg("tensor"), py::arg("root"),
           py::arg("op") = "sum", py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &dmp::RcclComm::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &dmp::RcclComm::reduce_scatter, py::arg("out"), py::arg("inp"),
           py::arg("op") = "sum", py::call_guard<py::gil_scoped_release>())
      .def("all_to_all", &dmp::RcclComm::all_to_all, py::call_guard<py::gil_scoped_release>())
      .def("send", &dmp::RcclComm::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &dmp::RcclComm::recv, py::call_guard<py::gil_scoped_release>())
      .def("batch_p2p", &dmp::RcclComm::batch_p2p, py::call_guard<py::gil_scoped_release>())
      .def("wait", &dmp::RcclComm::wait, py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &dmp::RcclComm::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("stream_handle",
           [](const dmp::RcclComm& c) { return reinterpret_cast<uintptr_t>(c.stream()); });

  // ---- DataParallel replica launcher ----
  py::class_<dmp::ParallelApply, std::shared_ptr<dmp::ParallelApply>>(m, "ParallelApply")
      .def(py::init<>())
      .def("apply", &dmp::ParallelApply::apply, py::arg("modules"), py::arg("inputs"),
           py::arg("kwargs"), py::arg("devices"), py::arg("streams") = std::vector<int64_t>{})
      .def("num_workers", &dmp::ParallelApply::num_workers)
      .def("last_times", &dmp::ParallelApply::last_times);

  // ---- DDP reducer ----
  py::class_<dmp::ReduceBackend, std::shared_ptr<dmp::ReduceBackend>>(m, "ReduceBackend");
  py::class_<dmp::RcclReduceBackend, dmp::ReduceBackend, std::shared_ptr<dmp::RcclReduceBackend>>(
      m, "RcclReduceBackend")
      .def(py::init<std::shared_ptr<dmp::RcclComm>, double, int64_t, bool>(), py::arg("comm"),
           py::arg("postscale") = 1.0, py::arg("debug_delay_cycles") = 0, py::arg("fp32_accum") = false)
      .def("set_timing", &dmp::RcclReduceBackend::set_timing, py::arg("on"))
      .def("last_timing", &dmp::RcclReduceBackend::last_timing,
           "[ready->done ms per bucket..., collective ms per bucket..., exposed tail ms] of the last backward",
           py::call_guard<py::gil_scoped_release>());
  py::class_<dmp::NullReduceBackend, dmp::ReduceBackend, std::shared_ptr<dmp::NullReduceBackend>>(
      m, "NullReduceBackend")
      .def(py::init<>());
  py::class_<dmp::PyReduceBackend, dmp::ReduceBackend, std::shared_ptr<dmp::PyReduceBackend>>(
      m, "PyReduceBackend")
      .def(py::init<py::object>());

  py::class_<dmp::Reducer, std::shared_ptr<dmp::Reducer>>(m, "Reducer")
      .def(py::init<std::vector<at::Tensor>, std::vector<std::vector<int64_t>>,
                    std::shared_ptr<dmp::ReduceBackend>, bool>(),
           py::arg("params"), py::arg("buckets"), py::arg("backend"), py::arg("find_unused"))
      .def("prepare_for_backward", &dmp::Reducer::prepare_for_backward,
           py::call_guard<py::gil_scoped_release>())
      .def("disarm", &dmp::Reducer::disarm)
      .def("rebuild", &dmp::Reducer::rebuild, py::call_guard<py::gil_scoped_release>())
      .def("buckets", &dmp::Reducer::buckets)
      .def("ready_order", &dmp::Reducer::ready_order)
      .def("group_flats", &dmp::Reducer::group_flats)
      .def("layout", &dmp::Reducer::layout)
      .def("grad_views", &dmp::Reducer::grad_views)
      .def("unused_params", &dmp::Reducer::unused_params)
      .def("num_launched", &dmp::Reducer::num_launched)
      .def("set_backend", &dmp::Reducer::set_backend)
      .def("zero_grad", &dmp::Reducer::zero_grad, py::call_guard<py::gil_scoped_release>());

  m.def("compute_bucket_assignment", &dmp::compute_bucket_assignment, py::arg("params"),
        py::arg("cap_bytes"), py::arg("first_cap_bytes"));
  // ops/wgrad_stream.py: which stream a leaf's AccumulateGrad node runs on
  // (-1: the leaf has no accumulator yet; -2: no accelerator stream)
  m.def("grad_accumulator_stream", [](const at::Tensor& t) -> int64_t {
    auto acc = torch::autograd::impl::try_get_grad_accumulator(t);
    if (!acc) return -1;
    auto s = acc->stream();
    return s.has_value() ? (int64_t)s->id() : -2;
  });
}
