// Operator schemas for torch.ops.llmctl.*  (implementations: TORCH_LIBRARY_IMPL(llmctl, CUDA)
// blocks in the individual .hip files; CUDA dispatch key == HIP on ROCm builds of PyTorch).
#include <torch/library.h>

namespace llmctl {  // custom_ar.hip: tensor-less helpers get catch-all kernels here
int64_t car_malloc(int64_t bytes);
void car_free(int64_t ptr);
at::Tensor car_ipc_handle(int64_t ptr);
int64_t car_ipc_open(const at::Tensor& handle);
void car_ipc_close(int64_t ptr);
int64_t car_sig_words();
int64_t car_error(int64_t sig_ptr);
void set_knob(const std::string& name, int64_t value);  // knobs.cpp
void clear_knobs();
}  // namespace llmctl

TORCH_LIBRARY(llmctl, m) {
  // norms (norm.hip)
  m.def("rmsnorm_fwd(Tensor x, Tensor w, float eps) -> (Tensor, Tensor)");
  m.def("add_rmsnorm_fwd(Tensor x, Tensor residual, Tensor w, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres) -> (Tensor, Tensor)");
  m.def("layernorm_fwd(Tensor x, Tensor w, Tensor b, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("add_layernorm_fwd(Tensor x, Tensor residual, Tensor w, Tensor b, float eps) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("layernorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor mu, Tensor rstd, Tensor? dres) -> (Tensor, Tensor, Tensor)");
  // elementwise (elementwise.hip)
  m.def("rope_qkv_fwd(Tensor qkv, Tensor cos, Tensor sin, int nq, int nkv, int seq_len, Tensor? positions) -> (Tensor, Tensor, Tensor)");
  m.def("rope_qk_inplace_(Tensor(a!) qkv, Tensor cos, Tensor sin, int nq, int nkv, int seq_len, Tensor? positions) -> ()");
  m.def("rope_qkv_cache_fwd(Tensor qkv, Tensor cos, Tensor sin, int nq, int nkv, int seq_len, Tensor? positions, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slots) -> (Tensor, Tensor, Tensor)");
  m.def("rope_qkv_bwd(Tensor dq, Tensor dk, Tensor dv, Tensor cos, Tensor sin, int seq_len, Tensor? positions) -> Tensor");
  m.def("swiglu_fwd(Tensor gu) -> Tensor");
  m.def("swiglu_bwd(Tensor dact, Tensor gu) -> Tensor");
  m.def("gelu_fwd(Tensor x) -> Tensor");
  m.def("gelu_bwd(Tensor dy, Tensor x) -> Tensor");
  // loss (loss.hip)
  m.def("cross_entropy_fwd(Tensor logits, Tensor labels, int ignore_index) -> (Tensor, Tensor)");
  m.def("cross_entropy_bwd(Tensor dloss, Tensor logits, Tensor lse, Tensor labels, int ignore_index, bool inplace) -> Tensor");
  // optimizer (optim.hip)
  m.def("adamw_step_(Tensor(a!) param, Tensor(b!) master, Tensor grad, Tensor(c!) exp_avg, Tensor(d!) exp_avg_sq, float lr, float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2, Tensor? grad_scale) -> ()");
  m.def("l2norm_sq_(Tensor x, Tensor(a!) out) -> ()");
  // attention (flash_attn_fwd.hip / flash_attn_bwd.hip)
  m.def("flash_attn_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal, Tensor? doc_start=None) -> (Tensor, Tensor)");
  m.def("flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, float scale, bool causal, Tensor? doc_start=None) -> (Tensor, Tensor, Tensor)");
  m.def("flash_attn_bwd_qkv(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, float scale, bool causal, Tensor? doc_start, Tensor cos, Tensor sin, Tensor? positions, int seq_len) -> Tensor");
  m.def("fa_bwd_ablate(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor delta, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, int abl) -> ()");
  // serving (paged_attn.hip, sampling.hip)
  m.def("kv_cache_write(Tensor k, Tensor v, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slot_mapping) -> ()");
  m.def("attn_merge_(Tensor(a!) o_acc, Tensor(b!) lse_acc, Tensor o_j, Tensor lse_j) -> ()");
  m.def("paged_prefill_attention(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor cu_q, Tensor ctx_lens, Tensor work, float scale) -> Tensor");
  m.def("paged_attention_decode(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor context_lens, float scale) -> Tensor");
  m.def("skinny_linear(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("skinny_linear_cfg(Tensor x, Tensor w, Tensor? bias, int config) -> Tensor");
  m.def("decode_qkv_rope_cache(Tensor x, Tensor w, Tensor? bias, Tensor cos, Tensor sin, int nq, int nkv, Tensor positions, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slots, Tensor? w_scale=None) -> Tensor");
  m.def("decode_up_swiglu(Tensor x, Tensor w, Tensor? bias, Tensor? w_scale=None) -> Tensor");
  m.def("decode_linear_partials(Tensor x, Tensor w, Tensor? w_scale=None) -> Tensor");
  m.def("decode_linear_add_rmsnorm(Tensor x, Tensor w, Tensor? bias, Tensor residual, Tensor norm_w, float eps, Tensor? w_scale=None) -> (Tensor, Tensor)");
  m.def("decode_linear_fp8(Tensor x, Tensor w, Tensor w_scale, Tensor? bias) -> Tensor");
  m.def("sample(Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor uniform) -> Tensor");
  // benchmarks / tuning (gemm_bf16.hip, hbm_stream.hip)
  m.def("gemm_bf16(Tensor a, Tensor b) -> Tensor");
  // custom all-reduce over xGMI peer memory (custom_ar.hip)
  m.def("car_allreduce(Tensor inp, Tensor(a!) out, Tensor data_ptrs, Tensor sig_ptrs, int rank, int world, int half_bytes) -> ()");
  m.def("car_allreduce_twoshot(Tensor inp, Tensor(a!) out, Tensor data_ptrs, Tensor sig_ptrs, int rank, int world, int half_bytes) -> ()");
  m.def("car_allreduce_add_rmsnorm(Tensor partial, Tensor? bias, Tensor res, Tensor nw, float eps, Tensor data_ptrs, Tensor sig_ptrs, int rank, int world, int half_bytes) -> (Tensor, Tensor)");
  m.def("car_malloc(int bytes) -> int", &llmctl::car_malloc);
  m.def("car_free(int ptr) -> ()", &llmctl::car_free);
  m.def("car_ipc_handle(int ptr) -> Tensor", &llmctl::car_ipc_handle);
  m.def("car_ipc_open(Tensor handle) -> int", &llmctl::car_ipc_open);
  m.def("car_ipc_close(int ptr) -> ()", &llmctl::car_ipc_close);
  m.def("car_sig_words() -> int", &llmctl::car_sig_words);
  m.def("car_error(int sig_ptr) -> int", &llmctl::car_error);
  m.def("set_knob(str name, int value) -> ()", &llmctl::set_knob);
  m.def("clear_knobs() -> ()", &llmctl::clear_knobs);
  m.def("gemm_ex(Tensor a, Tensor b, Tensor(a!) out, bool at, bool bt, bool accumulate, int variant=-1) -> ()");
  m.def("hbm_copy(Tensor src, Tensor(a!) dst) -> ()");
  m.def("gemm64_ex(Tensor a, Tensor b, Tensor(a!) out, bool at, bool bt, bool accumulate, int config=4) -> ()");
  m.def("gemm64_swiglu_fwd(Tensor x, Tensor w, int config, Tensor? rstd=None) -> Tensor");
  m.def("gemm64_rs(Tensor x, Tensor w, Tensor rstd, int config=304) -> Tensor");
  m.def("rms_rstd(Tensor x, float eps) -> Tensor");
  m.def("gemm64_swiglu_dgrad(Tensor dy, Tensor w, Tensor gu, int config=104) -> Tensor");
  m.def("gemm64_qkv_rope(Tensor x, Tensor w, Tensor cos, Tensor sin, Tensor? pos, int nq, int nkv, int seq, int config=104) -> (Tensor, Tensor, Tensor)");
  m.def("gemm64_up_swiglu(Tensor x, Tensor w, int config=104) -> (Tensor, Tensor)");
  m.def("gemm64_wgrad_swiglu(Tensor dy, Tensor act, Tensor(a!) gw, bool accumulate, Tensor dact, Tensor gu, int config=104) -> Tensor");
  m.def("transpose_(Tensor src, Tensor(a!) dst) -> ()");
}
