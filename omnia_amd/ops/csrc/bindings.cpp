// Python bindings for the omnia_amd gfx950 kernels.  Each entry validates the
// operand shapes/dtypes on the host BEFORE launching (a bad launch on the box
// can take every GPU of the host down), then launches on the current HIP
// stream so the calls are capturable into hipGraphs by the engine.
#include <chrono>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int omnia_pgemm(int epi, void* out, const void* X, const void* W, int M, int N, int K, int ldo,
                const float* ss_in, int ss_in_n, float inv_d, float eps, float* ss_out,
                const int* positions, const float* cos_sin, void* k_cache, void* v_cache,
                const int64_t* slots, int hq, int hkv, int block_size, hipStream_t s);
int omnia_row_sumsq(float* ss, const void* x, int rows, int d, int64_t stride, hipStream_t s);
int omnia_ar_alltoall(void* out, const void* in, void* const* regions, int* epochs, int* err,
                      int64_t chunk, int64_t slot_bytes, int rank, int world, hipStream_t s);
int omnia_ar_sendrecv(void* out, const void* in, void* const* regions, int* epochs, int* err,
                      int64_t nbytes, int64_t slot_bytes, int rank, int world, int src_rank,
                      hipStream_t s);
int omnia_pgemm_set_schedule(int sched);
int omnia_pgemm_splitk(void* parts, const void* X, const void* W, int M, int N, int K, int S,
                       int sched, hipStream_t s);
int omnia_pgemm_moe(int mode, void* out, const void* A, const void* W, const int* sorted,
                    const int* blk_expert, const int* n_blocks, const float* route_w, int K,
                    int N, int topk, int n_assign, int e_lo, int max_blocks, hipStream_t s);
int omnia_pgemm_variant(int variant, void* out, const void* X, const void* W, int M, int N,
                        int K, hipStream_t s);
int omnia_rmsnorm(void* out, const void* x, void* residual, const void* w, int rows, int d,
                  int64_t x_stride, int64_t out_stride, float eps, hipStream_t s);
int omnia_rope_kv(void* q, void* k, const void* v, const int* positions, const float* cos_sin,
                  void* k_cache, void* v_cache, const int64_t* slots, int T, int hq, int hkv,
                  int head_dim, int64_t q_stride, int64_t kv_stride, int block_size,
                  hipStream_t s);
int omnia_silu_mul(void* out, const void* x, int64_t T, int inter, hipStream_t s);
int omnia_embedding(void* out, const int* ids, const void* w, int T, int d, int vocab_start,
                    int vocab_end, const int64_t* src, const int* tok_slots, hipStream_t s);
int omnia_decode_attention(void* out, float* part_o, float* part_ml, const void* q,
                           const void* k_cache, const void* v_cache, const int* block_tables,
                           int bt_stride, const int* seq_lens, int B, int hq, int hkv,
                           int head_dim, int block_size, int64_t q_stride, int part_size,
                           int max_parts, float scale, int split_t, int split_min,
                           hipStream_t s);
int omnia_prefill_attention(void* out, const void* q, const void* k_cache, const void* v_cache,
                            const int* block_tables, int bt_stride, const int* q_start_loc,
                            const int* seq_lens, const int* tile_seq, const int* tile_q0,
                            int n_tiles, int hq, int hkv, int head_dim, int block_size,
                            int64_t q_stride, int64_t out_stride, float scale, int hp,
                            int q_tile, float* lse_out, const int* kv_lens, hipStream_t s);
int omnia_apply_token_mask(void* logits, int logits_is_bf16, int rows, int64_t row_stride,
                           int vocab, const uint32_t* mask, int words, hipStream_t s);
int omnia_sample(int* out_tok, float* out_logprob, const void* logits, int logits_is_bf16,
                 int rows, int64_t row_stride, int vocab, const float* temperature,
                 const int* top_k, const float* top_p, const uint64_t* seeds,
                 const int64_t* steps, int* counts, const float* freq_pen, const float* pres_pen,
                 const float* rep_pen, int* tok_slots, const int64_t* dst, hipStream_t s);
int omnia_tp_gumbel(float* pack, int64_t ld, int col, const void* logits, int rows,
                    int64_t row_stride, int vocab, int vocab_start, const float* temperature,
                    const int* top_k, const float* top_p, const int64_t* seeds,
                    const int64_t* steps, hipStream_t s);
int omnia_tp_pack(float* pack, int64_t ld, int K, const void* logits, int rows,
                  int64_t row_stride, int vocab, int vocab_start, const float* temperature,
                  const int* top_k, const float* top_p, const int64_t* seeds,
                  const int64_t* steps, hipStream_t s);
int omnia_tp_merge(int* out, int* tok_slots, const int64_t* dst_slot, const float* allp, int W,
                   int B, int64_t ld, int K, const float* temperature, const int* top_k,
                   const float* top_p, const int64_t* seeds, const int64_t* steps,
                   hipStream_t s);
int omnia_mean_pool_l2(float* out, const void* hidden, int64_t stride, const int* cu, int B,
                       int D, hipStream_t s);
int omnia_cosine_scores(float* scores, const float* q, int nq, const void* m, int64_t N, int D,
                        const uint8_t* valid, hipStream_t s);
int omnia_topk(int* out_idx, float* out_val, const float* scores, int nq, int64_t N, int k,
               hipStream_t s);
int omnia_moe_topk(int* ids, float* wts, const void* logits, int logits_bf16, int n_tok, int E,
                   int k, int renorm, hipStream_t s);
int omnia_moe_max_blocks(int n_assign, int n_experts, int bm);
int omnia_moe_router_topk(int* ids, float* wts, const void* x, const void* router, int n_tok,
                          int d, int E, int k, int renorm, hipStream_t s);
int omnia_moe_align(int* sorted, int* blk_expert, int* n_blocks, const int* ids, int n, int E,
                    int e_lo, int e_hi, int max_blocks, int bm, hipStream_t s);
int omnia_moe_gemm(int mode, void* out, const void* A, const void* W, const int* sorted,
                   const int* blk_expert, const int* n_blocks, const float* route_w, int K,
                   int N, int topk, int n_assign, int e_lo, int max_blocks, hipStream_t s);
int omnia_moe_combine(void* out, const void* Y, const int* ids, int n_tok, int d, int topk,
                      int e_lo, int e_hi, hipStream_t s);
int omnia_ipc_handle_size();
int omnia_ipc_alloc(void** ptr, int64_t bytes);
int omnia_ipc_free(void* ptr);
int omnia_ipc_get_handle(void* ptr, void* handle_out);
int omnia_ipc_open(const void* handle, void** ptr);
int omnia_ipc_close(void* ptr);
int omnia_ar_blocks();
int omnia_ar_max_ranks();
int omnia_ar_oneshot(void* out, const void* in, void* const* regions, int* epochs, int* err,
                     int64_t n, int64_t slot_bytes, int rank, int world, hipStream_t s);
int omnia_splitk_add_rmsnorm(void* out, const void* parts, int half, void* residual, const void* w, int S,
                             int M, int d, float eps, hipStream_t s);
int omnia_splitk_rope_kv(void* q, const void* parts, int half, int S, int T, const int* positions,
                         const float* cos_sin, void* k_cache, void* v_cache, const int64_t* slots,
                         int hq, int hkv, int head_dim, int block_size, hipStream_t s);
int omnia_splitk_swiglu(void* out, const void* parts, int half, int S, int M, int inter, hipStream_t s);
int omnia_splitk_reduce(void* out, const void* parts, int half, int S, int64_t n, hipStream_t s);
int64_t omnia_ar_region_bytes(int64_t slot_bytes);
int omnia_ar_twoshot(void* out, const void* in, void* residual, const void* w,
                     void* const* regions, int* epochs, int* err, int M, int d,
                     int64_t slot_bytes, int rank, int world, float eps, hipStream_t s);
int omnia_wgemm(int mode, void* out, const void* X, const void* W, int M, int N, int K, int S,
                int nw, int nwaves, int ldo, hipStream_t s);
int omnia_wgemm_wide(int mode, void* out, const void* X, const void* W, int M, int N, int K,
                     int S, int wt, int ldo, hipStream_t s);
int omnia_dgemm(int mode, void* out, const void* X, const void* W, float* ws, int* cnt, int M,
                int N, int K, int S, int wm, int wn, int ldo, int64_t ws_floats, int cnt_len,
                hipStream_t s);
int omnia_ar_allgather(void* out, const void* in, void* const* regions, int* epochs, int* err,
                       int64_t nbytes, int64_t slot_bytes, int rank, int world, hipStream_t s);
int omnia_tgemm(int mode, void* out, const void* X, const void* W, int M, int N, int K, int S,
                int bn, int wnt, int ldo, hipStream_t s);
int omnia_stage_copy(void* dst, const void* src, int64_t head_bytes, int64_t bt_off,
                     int64_t row_stride, int rows, int64_t row_bytes, hipStream_t s);
int64_t omnia_host_device_ptr(void* host);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_RC(rc, what) TORCH_CHECK((rc) == 0, what " launch failed rc=", (rc))

template <typename T>
T* opt_ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "rmsnorm expects 2-D");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1 && w.is_contiguous(), "inner dim contiguous");
  const int d = x.size(1);
  TORCH_CHECK(w.numel() == d && out.size(1) == d && out.size(0) == x.size(0), "shape mismatch");
  CHECK_RC(omnia_rmsnorm(out.data_ptr(), x.data_ptr(), nullptr, w.data_ptr(), x.size(0), d,
                         x.stride(0), out.stride(0), (float)eps, cur_stream()), "rmsnorm");
}

// residual += x ; x = rmsnorm(residual) * w      (both in place)
void fused_add_rmsnorm(at::Tensor x, at::Tensor residual, at::Tensor w, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && residual.is_contiguous(), "contiguous 2-D");
  TORCH_CHECK(residual.sizes() == x.sizes() && w.numel() == x.size(1), "shape mismatch");
  CHECK_RC(omnia_rmsnorm(x.data_ptr(), x.data_ptr(), residual.data_ptr(), w.data_ptr(),
                         x.size(0), x.size(1), x.stride(0), x.stride(0), (float)eps,
                         cur_stream()), "fused_add_rmsnorm");
}

void rope_kv(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor positions, at::Tensor cos_sin,
             c10::optional<at::Tensor> k_cache, c10::optional<at::Tensor> v_cache,
             c10::optional<at::Tensor> slots, int64_t hq, int64_t hkv, int64_t block_size) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_I32(positions);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous(), "cos_sin f32");
  TORCH_CHECK(q.dim() == 2 && k.dim() == 2 && v.dim() == 2, "q/k/v as [T, H*D] views");
  TORCH_CHECK(q.stride(1) == 1 && k.stride(1) == 1 && v.stride(1) == 1, "inner contiguous");
  TORCH_CHECK(k.stride(0) == v.stride(0), "k/v share row stride");
  const int T = q.size(0);
  const int D = q.size(1) / hq;
  TORCH_CHECK(D == 128 && k.size(1) == hkv * D && v.size(1) == hkv * D, "head_dim 128");
  TORCH_CHECK(positions.numel() == T && k.size(0) == T, "T mismatch");
  TORCH_CHECK(cos_sin.size(1) == D, "cos_sin width");
  const int64_t* sl = nullptr;
  void *kc = nullptr, *vc = nullptr;
  if (slots.has_value() && slots->defined()) {
    TORCH_CHECK(slots->scalar_type() == at::kLong && slots->numel() == T, "slots int64[T]");
    TORCH_CHECK(k_cache.has_value() && v_cache.has_value(), "caches required with slots");
    CHECK_BF16(*k_cache);
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == hkv && k_cache->size(2) == block_size &&
                k_cache->size(3) == D && k_cache->is_contiguous() && v_cache->is_contiguous(),
                "cache layout [NB, Hkv, BS, D]");
    sl = slots->data_ptr<int64_t>();
    kc = k_cache->data_ptr();
    vc = v_cache->data_ptr();
  }
  CHECK_RC(omnia_rope_kv(q.data_ptr(), k.data_ptr(), v.data_ptr(), positions.data_ptr<int>(),
                         cos_sin.data_ptr<float>(), kc, vc, sl, T, hq, hkv, D, q.stride(0),
                         k.stride(0), block_size, cur_stream()), "rope_kv");
}

void silu_mul(at::Tensor out, at::Tensor x) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(out);
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "contiguous");
  const int64_t inter = out.size(-1);
  TORCH_CHECK(x.size(-1) == 2 * inter && x.numel() == 2 * out.numel(), "shape mismatch");
  CHECK_RC(omnia_silu_mul(out.data_ptr(), x.data_ptr(), out.numel() / inter, inter,
                          cur_stream()), "silu_mul");
}

// src / tok_slots (optional, decode): row t's token is tok_slots[src[t]] when
// src[t] >= 0 (sampled on the device by an earlier step), else ids[t]
void embedding(at::Tensor out, at::Tensor ids, at::Tensor w, int64_t vocab_start,
               c10::optional<at::Tensor> src, c10::optional<at::Tensor> tok_slots) {
  CHECK_GPU(ids); CHECK_I32(ids); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(w.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(out.size(0) == ids.numel() && out.size(1) == w.size(1), "shape mismatch");
  const bool has_src = src.has_value() && src->defined();
  if (has_src) {
    CHECK_I32(*tok_slots);
    TORCH_CHECK(src->scalar_type() == at::kLong && src->numel() == ids.numel() &&
                src->is_contiguous() && tok_slots->is_contiguous(),
                "src [T] int64, tok_slots int32");
  }
  CHECK_RC(omnia_embedding(out.data_ptr(), ids.data_ptr<int>(), w.data_ptr(), ids.numel(),
                           w.size(1), vocab_start, vocab_start + w.size(0),
                           has_src ? src->data_ptr<int64_t>() : nullptr,
                           has_src ? tok_slots->data_ptr<int>() : nullptr, cur_stream()),
           "embedding");
}

void decode_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                      at::Tensor block_tables, at::Tensor seq_lens, at::Tensor part_o,
                      at::Tensor part_ml, int64_t part_size, double scale, int64_t splits,
                      int64_t split_min) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(seq_lens);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous(),
              "cache [NB, Hkv, BS, D]");
  const int hkv = k_cache.size(1), bs = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == D, "q [B, Hq, D]");
  const int B = q.size(0), hq = q.size(1);
  TORCH_CHECK(out.is_contiguous() && out.size(0) == B && out.size(1) == hq, "out [B, Hq, D]");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && block_tables.stride(1) == 1,
              "block_tables [B, max_blocks]");
  TORCH_CHECK(seq_lens.numel() >= B, "seq_lens");
  const int max_ctx = block_tables.size(1) * bs;
  // splits > 0: length-balanced split into up to `splits` partitions (>= split_min keys)
  TORCH_CHECK(splits >= 0 && (splits == 0 || split_min > 0), "splits / split_min");
  const int max_parts = std::max<int>((max_ctx + part_size - 1) / part_size, (int)splits);
  TORCH_CHECK(part_o.scalar_type() == at::kFloat && part_ml.scalar_type() == at::kFloat,
              "workspace f32");
  TORCH_CHECK(part_o.numel() >= (int64_t)B * hq * max_parts * D &&
              part_ml.numel() >= (int64_t)B * hq * max_parts * 2, "workspace too small");
  CHECK_RC(omnia_decode_attention(out.data_ptr(), part_o.data_ptr<float>(),
                                  part_ml.data_ptr<float>(), q.data_ptr(), k_cache.data_ptr(),
                                  v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                  block_tables.stride(0), seq_lens.data_ptr<int>(), B, hq, hkv, D,
                                  bs, q.stride(0), part_size, max_parts, (float)scale,
                                  (int)splits, (int)split_min, cur_stream()),
           "decode_attention");
}

void prefill_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                       at::Tensor block_tables, at::Tensor q_start_loc, at::Tensor seq_lens,
                       at::Tensor tile_seq, at::Tensor tile_q0, double scale, int64_t hp,
                       int64_t q_tile, c10::optional<at::Tensor> lse,
                       c10::optional<at::Tensor> kv_lens) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_BF16(k_cache);
  CHECK_I32(block_tables); CHECK_I32(q_start_loc); CHECK_I32(seq_lens); CHECK_I32(tile_seq);
  CHECK_I32(tile_q0);
  const int hkv = k_cache.size(1), bs = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == D, "q [T, Hq, D]");
  TORCH_CHECK(out.dim() == 3 && out.stride(2) == 1 && out.stride(1) == D, "out [T, Hq, D]");
  TORCH_CHECK(tile_seq.numel() == tile_q0.numel(), "tiles");
  TORCH_CHECK(block_tables.stride(1) == 1, "block_tables rows contiguous");
  float* lse_p = nullptr;
  if (lse.has_value()) {
    TORCH_CHECK(lse->scalar_type() == at::kFloat && lse->is_contiguous() && lse->dim() == 2 &&
                    lse->size(0) >= q.size(0) && lse->size(1) == q.size(1),
                "lse fp32 [T, Hq] contiguous");
    lse_p = lse->data_ptr<float>();
  }
  const int* kvl_p = nullptr;
  if (kv_lens.has_value()) {
    CHECK_I32((*kv_lens));
    TORCH_CHECK(kv_lens->numel() == seq_lens.numel(), "kv_lens [B]");
    kvl_p = kv_lens->data_ptr<int>();
  }
  CHECK_RC(omnia_prefill_attention(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(),
                                   v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                   block_tables.stride(0), q_start_loc.data_ptr<int>(),
                                   seq_lens.data_ptr<int>(), tile_seq.data_ptr<int>(),
                                   tile_q0.data_ptr<int>(), tile_seq.numel(), q.size(1), hkv, D,
                                   bs, q.stride(0), out.stride(0), (float)scale, (int)hp,
                                   (int)q_tile, lse_p, kvl_p, cur_stream()),
           "prefill_attention");
}

void sample(at::Tensor out_tok, c10::optional<at::Tensor> out_logprob, at::Tensor logits,
            at::Tensor temperature, c10::optional<at::Tensor> top_k,
            c10::optional<at::Tensor> top_p, c10::optional<at::Tensor> seeds,
            c10::optional<at::Tensor> steps, c10::optional<at::Tensor> counts,
            c10::optional<at::Tensor> freq_pen, c10::optional<at::Tensor> pres_pen,
            c10::optional<at::Tensor> rep_pen, c10::optional<at::Tensor> tok_slots,
            c10::optional<at::Tensor> dst) {
  CHECK_GPU(logits); CHECK_I32(out_tok);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V]");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat,
              "logits bf16/f32");
  const int rows = logits.size(0), vocab = logits.size(1);
  TORCH_CHECK(out_tok.numel() >= rows && temperature.numel() >= rows, "per-row params");
  if (counts.has_value() && counts->defined())
    TORCH_CHECK(counts->scalar_type() == at::kInt && counts->size(0) >= rows &&
                counts->size(1) == vocab && counts->is_contiguous(), "counts int32 [B, V]");
  if (tok_slots.has_value() && tok_slots->defined()) {
    CHECK_I32(*tok_slots);
    TORCH_CHECK(dst.has_value() && dst->defined() && dst->scalar_type() == at::kLong &&
                dst->numel() >= rows && dst->is_contiguous() && tok_slots->is_contiguous(),
                "tok_slots int32 + dst int64 [B]");
  }
  CHECK_RC(omnia_sample(out_tok.data_ptr<int>(), opt_ptr<float>(out_logprob), logits.data_ptr(),
                        logits.scalar_type() == at::kBFloat16, rows, logits.stride(0), vocab,
                        temperature.data_ptr<float>(), opt_ptr<int>(top_k), opt_ptr<float>(top_p),
                        opt_ptr<uint64_t>(seeds), opt_ptr<int64_t>(steps), opt_ptr<int>(counts),
                        opt_ptr<float>(freq_pen), opt_ptr<float>(pres_pen),
                        opt_ptr<float>(rep_pen), opt_ptr<int>(tok_slots), opt_ptr<int64_t>(dst),
                        cur_stream()), "sample");
}

// K13: grammar mask -> -inf logits (mask int32 [rows, ceil(V/32)], bit v = allowed)
// TP sampling: per-row Gumbel-max winner of this rank's vocab slice, written
// into columns col, col+1 of the fp32 candidate pack [B, ld]
void tp_gumbel(at::Tensor pack, int64_t col, at::Tensor logits, int64_t vocab_start,
               at::Tensor temperature, c10::optional<at::Tensor> top_k,
               c10::optional<at::Tensor> top_p, at::Tensor seeds,
               c10::optional<at::Tensor> steps) {
  CHECK_GPU(pack); CHECK_GPU(logits); CHECK_BF16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V] inner-contiguous");
  const int rows = logits.size(0), vocab = logits.size(1);
  TORCH_CHECK(pack.scalar_type() == at::kFloat && pack.dim() == 2 && pack.stride(1) == 1 &&
              pack.size(0) == rows && col >= 0 && col + 2 <= pack.size(1), "pack fp32 [B, ld]");
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && temperature.numel() >= rows &&
              temperature.is_cuda(), "temperature fp32 [B]");
  TORCH_CHECK(seeds.scalar_type() == at::kLong && seeds.numel() >= rows && seeds.is_cuda(),
              "seeds int64 [B]");
  if (top_k.has_value() && top_k->defined())
    TORCH_CHECK(top_k->scalar_type() == at::kInt && top_k->numel() >= rows, "top_k int32 [B]");
  if (top_p.has_value() && top_p->defined())
    TORCH_CHECK(top_p->scalar_type() == at::kFloat && top_p->numel() >= rows, "top_p fp32 [B]");
  if (steps.has_value() && steps->defined())
    TORCH_CHECK(steps->scalar_type() == at::kLong && steps->numel() >= rows, "steps int64 [B]");
  CHECK_RC(omnia_tp_gumbel(pack.data_ptr<float>(), pack.stride(0), (int)col, logits.data_ptr(),
                           rows, logits.stride(0), vocab, (int)vocab_start,
                           temperature.data_ptr<float>(), opt_ptr<int>(top_k),
                           opt_ptr<float>(top_p), seeds.data_ptr<int64_t>(),
                           opt_ptr<int64_t>(steps), cur_stream()), "tp_gumbel");
}

// TP sampler, per rank: candidate pack of this rank's vocab slice (sampling.hip)
void tp_pack(at::Tensor pack, int64_t K, at::Tensor logits, int64_t vocab_start,
             at::Tensor temperature, c10::optional<at::Tensor> top_k,
             c10::optional<at::Tensor> top_p, at::Tensor seeds, c10::optional<at::Tensor> steps) {
  CHECK_GPU(pack); CHECK_GPU(logits); CHECK_BF16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V] inner-contiguous");
  const int rows = logits.size(0), vocab = logits.size(1);
  TORCH_CHECK(pack.scalar_type() == at::kFloat && pack.dim() == 2 && pack.is_contiguous() &&
              pack.size(0) == rows && pack.size(1) >= 2 * K + 4 && K >= 1 && K <= vocab,
              "pack fp32 [B, >= 2K+4] contiguous, 1 <= K <= V");
  TORCH_CHECK(temperature.is_cuda() && temperature.scalar_type() == at::kFloat &&
              temperature.numel() >= rows, "temperature fp32 [B]");
  TORCH_CHECK(seeds.is_cuda() && seeds.scalar_type() == at::kLong && seeds.numel() >= rows,
              "seeds int64 [B]");
  if (top_k.has_value() && top_k->defined())
    TORCH_CHECK(top_k->is_cuda() && top_k->scalar_type() == at::kInt && top_k->numel() >= rows,
                "top_k int32 [B]");
  if (top_p.has_value() && top_p->defined())
    TORCH_CHECK(top_p->is_cuda() && top_p->scalar_type() == at::kFloat && top_p->numel() >= rows,
                "top_p fp32 [B]");
  if (steps.has_value() && steps->defined())
    TORCH_CHECK(steps->is_cuda() && steps->scalar_type() == at::kLong && steps->numel() >= rows,
                "steps int64 [B]");
  CHECK_RC(omnia_tp_pack(pack.data_ptr<float>(), pack.stride(0), (int)K, logits.data_ptr(), rows,
                         logits.stride(0), vocab, (int)vocab_start, temperature.data_ptr<float>(),
                         opt_ptr<int>(top_k), opt_ptr<float>(top_p), seeds.data_ptr<int64_t>(),
                         opt_ptr<int64_t>(steps), cur_stream()), "tp_pack");
}

// TP sampler, every rank: token of each row from the all-gathered packs [W, B, ld];
// with tok_slots / dst, also tok_slots[dst[r]] = token (device token hand-off)
void tp_merge(at::Tensor out, c10::optional<at::Tensor> tok_slots, c10::optional<at::Tensor> dst,
              at::Tensor allp, int64_t K, at::Tensor temperature, c10::optional<at::Tensor> top_k,
              c10::optional<at::Tensor> top_p, at::Tensor seeds, c10::optional<at::Tensor> steps) {
  CHECK_GPU(out); CHECK_GPU(allp); CHECK_I32(out);
  TORCH_CHECK(allp.scalar_type() == at::kFloat && allp.dim() == 3 && allp.is_contiguous(),
              "allp fp32 [W, B, ld] contiguous");
  const int W = allp.size(0), B = allp.size(1);
  const int64_t ld = allp.size(2);
  TORCH_CHECK(out.numel() >= B && out.is_contiguous(), "out int32 [B]");
  TORCH_CHECK(K >= 1 && ld >= 2 * K + 4 && W * K <= 512, "W * K <= 512, ld >= 2K+4");
  TORCH_CHECK(temperature.is_cuda() && temperature.scalar_type() == at::kFloat &&
              temperature.numel() >= B, "temperature fp32 [B]");
  TORCH_CHECK(seeds.is_cuda() && seeds.scalar_type() == at::kLong && seeds.numel() >= B,
              "seeds int64 [B]");
  if (top_k.has_value() && top_k->defined())
    TORCH_CHECK(top_k->scalar_type() == at::kInt && top_k->numel() >= B, "top_k int32 [B]");
  if (top_p.has_value() && top_p->defined())
    TORCH_CHECK(top_p->scalar_type() == at::kFloat && top_p->numel() >= B, "top_p fp32 [B]");
  if (steps.has_value() && steps->defined())
    TORCH_CHECK(steps->scalar_type() == at::kLong && steps->numel() >= B, "steps int64 [B]");
  const bool slots = tok_slots.has_value() && tok_slots->defined();
  if (slots) {
    TORCH_CHECK(dst.has_value() && dst->defined() && dst->scalar_type() == at::kLong &&
                dst->numel() >= B && dst->is_cuda(), "dst int64 [B] with tok_slots");
    CHECK_I32(*tok_slots);
    TORCH_CHECK(tok_slots->is_cuda() && tok_slots->is_contiguous(), "tok_slots int32 on device");
  }
  CHECK_RC(omnia_tp_merge(out.data_ptr<int>(), slots ? tok_slots->data_ptr<int>() : nullptr,
                          slots ? dst->data_ptr<int64_t>() : nullptr, allp.data_ptr<float>(), W, B,
                          ld, (int)K, temperature.data_ptr<float>(), opt_ptr<int>(top_k),
                          opt_ptr<float>(top_p), seeds.data_ptr<int64_t>(),
                          opt_ptr<int64_t>(steps), cur_stream()), "tp_merge");
}

void apply_token_mask(at::Tensor logits, at::Tensor mask) {
  CHECK_GPU(logits); CHECK_GPU(mask); CHECK_I32(mask);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V]");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat,
              "logits bf16/f32");
  const int rows = logits.size(0), vocab = logits.size(1), words = (vocab + 31) / 32;
  TORCH_CHECK(mask.dim() == 2 && mask.size(0) == rows && mask.size(1) == words &&
              mask.is_contiguous(), "mask int32 [B, ceil(V/32)] contiguous");
  CHECK_RC(omnia_apply_token_mask(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, rows,
                                  logits.stride(0), vocab,
                                  reinterpret_cast<const uint32_t*>(mask.data_ptr<int>()), words,
                                  cur_stream()), "apply_token_mask");
}

// K17: out[b] = normalize(mean(hidden[cu[b]:cu[b+1]]))   fp32
void mean_pool_l2(at::Tensor out, at::Tensor hidden, at::Tensor cu) {
  CHECK_GPU(hidden); CHECK_BF16(hidden); CHECK_I32(cu);
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous(), "out fp32 contiguous");
  TORCH_CHECK(hidden.dim() == 2 && hidden.stride(1) == 1, "hidden [T, D] inner-contiguous");
  TORCH_CHECK(cu.dim() == 1 && cu.is_contiguous() && cu.is_cuda(), "cu [B+1] on device");
  const int B = cu.size(0) - 1, D = hidden.size(1);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == B && out.size(1) == D, "out [B, D]");
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "D must be a multiple of 8, <= 8192");
  CHECK_RC(omnia_mean_pool_l2(out.data_ptr<float>(), hidden.data_ptr(), hidden.stride(0),
                              cu.data_ptr<int>(), B, D, cur_stream()), "mean_pool_l2");
}

// K18: scores[q, n] = Q[q] . M[n]  (fp32 out, -inf where valid[n] == 0)
void cosine_scores(at::Tensor scores, at::Tensor q, at::Tensor m,
                   c10::optional<at::Tensor> valid) {
  CHECK_GPU(m); CHECK_BF16(m);
  TORCH_CHECK(q.scalar_type() == at::kFloat && q.is_contiguous() && q.is_cuda(), "q fp32");
  TORCH_CHECK(m.dim() == 2 && m.is_contiguous(), "m [N, D] contiguous");
  TORCH_CHECK(q.dim() == 2 && q.size(1) == m.size(1), "q [NQ, D]");
  const int nq = q.size(0), D = m.size(1);
  const int64_t N = m.size(0);
  TORCH_CHECK(nq == 1 || nq == 2 || nq == 4 || nq == 8, "NQ must be 1/2/4/8 (pad on host)");
  TORCH_CHECK((int64_t)nq * D * 4 <= 64 * 1024, "NQ*D too large for the LDS stage");
  TORCH_CHECK(D % 8 == 0, "D % 8");
  TORCH_CHECK(scores.scalar_type() == at::kFloat && scores.is_contiguous() &&
              scores.size(0) == nq && scores.size(1) == N, "scores [NQ, N] fp32");
  const uint8_t* vp = nullptr;
  if (valid.has_value() && valid->defined()) {
    TORCH_CHECK(valid->scalar_type() == at::kByte && valid->numel() >= N && valid->is_cuda(),
                "valid uint8 [>= N]");
    vp = valid->data_ptr<uint8_t>();
  }
  CHECK_RC(omnia_cosine_scores(scores.data_ptr<float>(), q.data_ptr<float>(), nq, m.data_ptr(),
                               N, D, vp, cur_stream()), "cosine_scores");
}

void topk(at::Tensor out_idx, at::Tensor out_val, at::Tensor scores, int64_t k) {
  CHECK_GPU(scores);
  TORCH_CHECK(scores.scalar_type() == at::kFloat && scores.is_contiguous() && scores.dim() == 2,
              "scores [NQ, N] fp32 contiguous");
  const int nq = scores.size(0);
  const int64_t N = scores.size(1);
  TORCH_CHECK(k >= 1 && k <= 1024 && k <= N, "1 <= k <= min(1024, N)");
  CHECK_I32(out_idx);
  TORCH_CHECK(out_val.scalar_type() == at::kFloat, "out_val fp32");
  TORCH_CHECK(out_idx.numel() == nq * k && out_val.numel() == nq * k && out_idx.is_contiguous() &&
              out_val.is_contiguous(), "outputs [NQ, k]");
  CHECK_RC(omnia_topk(out_idx.data_ptr<int>(), out_val.data_ptr<float>(),
                      scores.data_ptr<float>(), nq, N, (int)k, cur_stream()), "topk");
}

// ---------------------------------------------------------------- MoE (K14)
void moe_topk(at::Tensor ids, at::Tensor wts, at::Tensor logits, int64_t k, bool renorm) {
  CHECK_GPU(logits); CHECK_I32(ids);
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits [T, E] contiguous");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "logits bf16/fp32");
  const int T = logits.size(0), E = logits.size(1);
  TORCH_CHECK(E <= 64 && k >= 1 && k <= E, "E <= 64, 1 <= k <= E");
  TORCH_CHECK(ids.numel() == (int64_t)T * k && wts.numel() == (int64_t)T * k &&
              wts.scalar_type() == at::kFloat && ids.is_contiguous() && wts.is_contiguous(),
              "ids/wts [T, k]");
  CHECK_RC(omnia_moe_topk(ids.data_ptr<int>(), wts.data_ptr<float>(), logits.data_ptr(), bf, T,
                          E, k, renorm, cur_stream()), "moe_topk");
}

// router GEMM + top-k in one kernel: x [T, d] bf16, router [E, d] bf16 -> ids / wts [T, k]
void moe_router_topk(at::Tensor ids, at::Tensor wts, at::Tensor x, at::Tensor router, int64_t k,
                     bool renorm) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(router); CHECK_I32(ids);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && router.dim() == 2 && router.is_contiguous() &&
              router.size(1) == x.size(1) && x.size(1) % 8 == 0, "x [T, d], router [E, d]");
  const int T = x.size(0), E = router.size(0);
  TORCH_CHECK(E <= 64 && k >= 1 && k <= E, "E <= 64, 1 <= k <= E");
  TORCH_CHECK(ids.numel() == (int64_t)T * k && wts.numel() == (int64_t)T * k &&
              wts.scalar_type() == at::kFloat && ids.is_contiguous() && wts.is_contiguous(),
              "ids/wts [T, k]");
  CHECK_RC(omnia_moe_router_topk(ids.data_ptr<int>(), wts.data_ptr<float>(), x.data_ptr(),
                                 router.data_ptr(), T, x.size(1), E, k, renorm, cur_stream()),
           "moe_router_topk");
}

int64_t moe_max_blocks(int64_t n_assign, int64_t n_experts, int64_t bm) {
  return omnia_moe_max_blocks(n_assign, n_experts, bm);
}

// segments aligned to bm = sorted.numel() / blk_expert.numel() rows (64: moe_gemm,
// 256: the pgemm_moe prefill tile)
void moe_align(at::Tensor sorted, at::Tensor blk_expert, at::Tensor n_blocks, at::Tensor ids,
               int64_t E, int64_t e_lo, int64_t e_hi) {
  CHECK_GPU(ids); CHECK_I32(ids); CHECK_I32(sorted); CHECK_I32(blk_expert); CHECK_I32(n_blocks);
  const int n = ids.numel();
  const int mb = blk_expert.numel();
  TORCH_CHECK(mb > 0 && (sorted.numel() == (int64_t)mb * 64 || sorted.numel() == (int64_t)mb * 256),
              "sorted must hold max_blocks*64 (or *256) rows");
  const int bm = (int)(sorted.numel() / mb);
  TORCH_CHECK(mb >= omnia_moe_max_blocks(n, e_hi - e_lo, bm), "blk_expert too small");
  TORCH_CHECK(E <= 256 && 0 <= e_lo && e_lo < e_hi && e_hi <= E, "expert range");
  CHECK_RC(omnia_moe_align(sorted.data_ptr<int>(), blk_expert.data_ptr<int>(),
                           n_blocks.data_ptr<int>(), ids.data_ptr<int>(), n, E, e_lo, e_hi, mb,
                           bm, cur_stream()), "moe_align");
}

// the 256x256-tile grouped MoE GEMMs (pgemm.hip EPI 5 / 6) over 256-row segments
void pgemm_moe(int64_t mode, at::Tensor out, at::Tensor A, at::Tensor W, at::Tensor sorted,
               at::Tensor blk_expert, at::Tensor n_blocks, c10::optional<at::Tensor> route_w,
               int64_t topk, int64_t n_assign, int64_t e_lo) {
  CHECK_GPU(A); CHECK_BF16(A); CHECK_BF16(W); CHECK_BF16(out);
  CHECK_I32(sorted); CHECK_I32(blk_expert); CHECK_I32(n_blocks);
  TORCH_CHECK(A.is_contiguous() && W.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(W.dim() == 3, "W [E_local, rows, K]");
  const int K = W.size(2);
  const int mb = blk_expert.numel();
  TORCH_CHECK(sorted.numel() == (int64_t)mb * 256, "sorted must hold max_blocks*256 rows");
  TORCH_CHECK(A.size(-1) == K && K % 128 == 0, "K mismatch / K % 128");
  int N;
  if (mode == 0) {
    N = W.size(1) / 2;
    TORCH_CHECK(N % 128 == 0 && out.size(0) == (int64_t)mb * 256 && out.size(1) == N,
                "act [max_blocks*256, I]");
    TORCH_CHECK(A.size(0) * topk == n_assign, "x rows * topk == n_assign");
  } else {
    N = W.size(1);
    TORCH_CHECK(N % 256 == 0 && out.size(0) == n_assign && out.size(1) == N, "Y [T*k, d]");
    TORCH_CHECK(A.size(0) == (int64_t)mb * 256, "act rows");
    TORCH_CHECK(route_w.has_value() && route_w->numel() == n_assign &&
                route_w->scalar_type() == at::kFloat, "route weights");
  }
  CHECK_RC(omnia_pgemm_moe((int)mode, out.data_ptr(), A.data_ptr(), W.data_ptr(),
                           sorted.data_ptr<int>(), blk_expert.data_ptr<int>(),
                           n_blocks.data_ptr<int>(), opt_ptr<float>(route_w), K, N, topk,
                           n_assign, e_lo, mb, cur_stream()), "pgemm_moe");
}

void moe_gemm(int64_t mode, at::Tensor out, at::Tensor A, at::Tensor W, at::Tensor sorted,
              at::Tensor blk_expert, at::Tensor n_blocks, c10::optional<at::Tensor> route_w,
              int64_t topk, int64_t n_assign, int64_t e_lo) {
  CHECK_GPU(A); CHECK_BF16(A); CHECK_BF16(W); CHECK_BF16(out);
  TORCH_CHECK(A.is_contiguous() && W.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(W.dim() == 3, "W [E_local, rows, K]");
  const int K = W.size(2);
  const int mb = blk_expert.numel();
  TORCH_CHECK(A.size(-1) == K && K % 64 == 0, "K mismatch / K % 64");
  int N;
  if (mode == 0) {
    N = W.size(1) / 2;
    TORCH_CHECK(N % 32 == 0 && out.size(0) == (int64_t)mb * 64 && out.size(1) == N,
                "act [max_blocks*64, I]");
    TORCH_CHECK(A.size(0) * topk == n_assign, "x rows * topk == n_assign");
  } else {
    N = W.size(1);
    TORCH_CHECK(N % 64 == 0 && out.size(0) == n_assign && out.size(1) == N, "Y [T*k, d]");
    TORCH_CHECK(A.size(0) == (int64_t)mb * 64, "act rows");
    TORCH_CHECK(route_w.has_value() && route_w->numel() == n_assign, "route weights");
  }
  CHECK_RC(omnia_moe_gemm((int)mode, out.data_ptr(), A.data_ptr(), W.data_ptr(),
                          sorted.data_ptr<int>(), blk_expert.data_ptr<int>(),
                          n_blocks.data_ptr<int>(), opt_ptr<float>(route_w), K, N, topk,
                          n_assign, e_lo, mb, cur_stream()), "moe_gemm");
}

void moe_combine(at::Tensor out, at::Tensor Y, at::Tensor ids, int64_t topk, int64_t e_lo,
                 int64_t e_hi) {
  CHECK_GPU(Y); CHECK_BF16(Y); CHECK_BF16(out); CHECK_I32(ids);
  const int T = out.size(0), d = out.size(1);
  TORCH_CHECK(Y.size(0) == (int64_t)T * topk && Y.size(1) == d && ids.numel() == T * topk,
              "Y [T*k, d]");
  CHECK_RC(omnia_moe_combine(out.data_ptr(), Y.data_ptr(), ids.data_ptr<int>(), T, d, topk,
                             e_lo, e_hi, cur_stream()), "moe_combine");
}

// decode projection GEMM: mode 0 out[M,N] = x W^T (W [N,K]); mode 1 out[M,I] =
// silu(x Wg^T) * (x Wu^T) with W = [Wg; Wu] ([2I, K]).  Shapes are validated
// here AND in omnia_dgemm before anything is launched.
void dgemm(int64_t mode, at::Tensor out, at::Tensor x, at::Tensor W, at::Tensor ws, at::Tensor cnt,
           int64_t splits, int64_t wm, int64_t wn) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(W); CHECK_BF16(out);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_cuda(), "ws fp32");
  CHECK_I32(cnt);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && out.dim() == 2, "2-D operands");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous() && out.stride(1) == 1, "contiguous");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(W.size(1) == K, "K mismatch");
  const int N = mode == 0 ? W.size(0) : W.size(0) / 2;
  TORCH_CHECK(mode == 0 || W.size(0) % 2 == 0, "gate_up rows even");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "out shape");
  CHECK_RC(omnia_dgemm((int)mode, out.data_ptr(), x.data_ptr(), W.data_ptr(),
                       ws.data_ptr<float>(), cnt.data_ptr<int>(), M, N, K, (int)splits, (int)wm,
                       (int)wn, (int)out.stride(0), ws.numel(), (int)cnt.numel(), cur_stream()),
           "dgemm");
}

// weight-streaming decode GEMM (wgemm.hip): mode 0 bf16 out[M,N] = x W^T; mode 1
// SwiGLU bf16 out[M,I] from W = [Wg; Wu]; mode 2 fp32 split-K slabs out[S,M,N].
void wgemm(int64_t mode, at::Tensor out, at::Tensor x, at::Tensor W, int64_t splits, int64_t nw,
           int64_t nwaves) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(W);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2, "2-D operands");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous(), "contiguous x / W");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(W.size(1) == K, "K mismatch");
  TORCH_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  TORCH_CHECK(mode != 1 || W.size(0) % 2 == 0, "gate_up rows even");
  const int N = mode == 1 ? W.size(0) / 2 : W.size(0);
  int ldo;
  if (mode == 2) {
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_cuda() && out.is_contiguous(),
                "mode 2: fp32 contiguous slabs");
    TORCH_CHECK(out.dim() == 3 && out.size(0) == splits && out.size(1) == M && out.size(2) == N,
                "mode 2: out [S, M, N]");
    ldo = N;
  } else {
    CHECK_BF16(out);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1,
                "out [M, N]");
    ldo = out.stride(0);
  }
  CHECK_RC(omnia_wgemm((int)mode, out.data_ptr(), x.data_ptr(), W.data_ptr(), M, N, K,
                       (int)splits, (int)nw, (int)nwaves, ldo, cur_stream()),
           "wgemm");
}

// wide-batch weight-streaming decode GEMM (wgemm_wide.hip, 128 < M <= 256):
// same modes / out shapes as wgemm; wt = 32-column MFMA tiles per wave (1 or 2)
void wgemm_wide(int64_t mode, at::Tensor out, at::Tensor x, at::Tensor W, int64_t splits,
                int64_t wt) {
  CHECK_BF16(x); CHECK_BF16(W);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2, "2-D operands");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous(), "contiguous x / W");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(W.size(1) == K, "K mismatch");
  TORCH_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  TORCH_CHECK(mode != 1 || W.size(0) % 2 == 0, "gate_up rows even");
  const int N = mode == 1 ? W.size(0) / 2 : W.size(0);
  int ldo;
  if (mode == 2) {
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_cuda() && out.is_contiguous(),
                "mode 2: fp32 contiguous slabs");
    TORCH_CHECK(out.dim() == 3 && out.size(0) == splits && out.size(1) == M && out.size(2) == N,
                "mode 2: out [S, M, N]");
    ldo = N;
  } else {
    CHECK_BF16(out);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1,
                "out [M, N]");
    ldo = out.stride(0);
  }
  CHECK_RC(omnia_wgemm_wide((int)mode, out.data_ptr(), x.data_ptr(), W.data_ptr(), M, N, K,
                            (int)splits, (int)wt, ldo, cur_stream()),
           "wgemm_wide");
}

// full-batch tile decode GEMM (tgemm.hip, M <= 256): same modes / out shapes as
// wgemm; bn = weight rows per block (64/128/256), wnt = non-temporal weight loads
void tgemm(int64_t mode, at::Tensor out, at::Tensor x, at::Tensor W, int64_t splits, int64_t bn,
           int64_t wnt) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(W);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2, "2-D operands");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous(), "contiguous x / W");
  TORCH_CHECK(x.device() == W.device() && x.device() == out.device(), "same device");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(W.size(1) == K, "K mismatch");
  TORCH_CHECK(mode >= 0 && mode <= 3, "mode");
  TORCH_CHECK(mode != 1 || W.size(0) % 2 == 0, "gate_up rows even");
  const int N = mode == 1 ? W.size(0) / 2 : W.size(0);
  int ldo;
  if (mode >= 2) {
    TORCH_CHECK(out.scalar_type() == (mode == 2 ? at::kFloat : at::kHalf) && out.is_contiguous(),
                "mode 2 / 3: fp32 / fp16 contiguous slabs");
    TORCH_CHECK(out.dim() == 3 && out.size(0) == splits && out.size(1) == M && out.size(2) == N,
                "mode 2 / 3: out [S, M, N]");
    ldo = N;
  } else {
    CHECK_BF16(out);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1,
                "out [M, N]");
    ldo = out.stride(0);
  }
  CHECK_RC(omnia_tgemm((int)mode, out.data_ptr(), x.data_ptr(), W.data_ptr(), M, N, K,
                       (int)splits, (int)bn, (int)wnt, ldo, cur_stream()),
           "tgemm");
}

// prefill GEMM with fused epilogues (pgemm.hip, 256x256 tiles): epi 0 plain
// (optionally row-scaled), 1 gate_up + SwiGLU, 2 residual add + row sum of
// squares, 3 QKV + RoPE + paged KV write.  ss_in = partial row sums of squares
// [M, n] of x (row scale rsqrt(sum / d + eps)), ss_out = [M, N / 256].
void pgemm(int64_t epi, at::Tensor out, at::Tensor x, at::Tensor W,
           c10::optional<at::Tensor> ss_in, double inv_d, double eps,
           c10::optional<at::Tensor> ss_out, c10::optional<at::Tensor> positions,
           c10::optional<at::Tensor> cos_sin, c10::optional<at::Tensor> k_cache,
           c10::optional<at::Tensor> v_cache, c10::optional<at::Tensor> slots, int64_t hq,
           int64_t hkv, int64_t block_size) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(W); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && out.dim() == 2, "2-D operands");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous(), "contiguous x / W");
  TORCH_CHECK(out.stride(1) == 1, "out rows contiguous");
  TORCH_CHECK(x.device() == W.device() && x.device() == out.device(), "same device");
  TORCH_CHECK(epi >= 0 && epi <= 3, "epi");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(W.size(1) == K, "K mismatch");
  TORCH_CHECK(epi != 1 || W.size(0) % 2 == 0, "gate_up rows even");
  const int N = epi == 1 ? W.size(0) / 2 : W.size(0);
  TORCH_CHECK(out.size(0) == M, "out rows");
  TORCH_CHECK(out.size(1) == (epi == 3 ? hq * 128 : N), "out [M, N] (q [M, hq*128] for epi 3)");
  const float* ssi = nullptr;
  int ssn = 0;
  if (ss_in.has_value() && ss_in->defined()) {
    TORCH_CHECK(ss_in->scalar_type() == at::kFloat && ss_in->is_contiguous() && ss_in->dim() == 2 &&
                ss_in->size(0) == M && ss_in->device() == x.device(), "ss_in fp32 [M, n]");
    ssi = ss_in->data_ptr<float>();
    ssn = ss_in->size(1);
  }
  float* sso = nullptr;
  if (epi == 2) {
    TORCH_CHECK(ss_out.has_value() && ss_out->defined(), "epi 2 needs ss_out");
    TORCH_CHECK(ss_out->scalar_type() == at::kFloat && ss_out->is_contiguous() &&
                ss_out->dim() == 2 && ss_out->size(0) == M && ss_out->size(1) == N / 256 &&
                ss_out->device() == x.device(), "ss_out fp32 [M, N/256]");
    sso = ss_out->data_ptr<float>();
  }
  const int* pos = nullptr;
  const float* cs = nullptr;
  void *kc = nullptr, *vc = nullptr;
  const int64_t* sl = nullptr;
  if (epi == 3) {
    TORCH_CHECK(positions.has_value() && cos_sin.has_value() && k_cache.has_value() &&
                v_cache.has_value() && slots.has_value(), "epi 3 needs rope / cache operands");
    TORCH_CHECK(positions->scalar_type() == at::kInt && positions->numel() == M &&
                positions->is_contiguous(), "positions int32 [M]");
    TORCH_CHECK(cos_sin->scalar_type() == at::kFloat && cos_sin->is_contiguous() &&
                cos_sin->dim() == 2 && cos_sin->size(1) == 128, "cos_sin f32 [P, 128]");
    TORCH_CHECK(slots->scalar_type() == at::kLong && slots->numel() == M && slots->is_contiguous(),
                "slots int64 [M]");
    CHECK_BF16(*k_cache); CHECK_BF16(*v_cache);
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == hkv && k_cache->size(2) == block_size &&
                k_cache->size(3) == 128 && k_cache->is_contiguous() && v_cache->is_contiguous() &&
                v_cache->sizes() == k_cache->sizes(), "cache layout [NB, Hkv, BS, 128]");
    for (const at::Tensor* t : {&*positions, &*cos_sin, &*k_cache, &*v_cache, &*slots})
      TORCH_CHECK(t->device() == x.device(), "same device");
    pos = positions->data_ptr<int>();
    cs = cos_sin->data_ptr<float>();
    kc = k_cache->data_ptr();
    vc = v_cache->data_ptr();
    sl = slots->data_ptr<int64_t>();
  }
  if (M == 0) return;
  CHECK_RC(omnia_pgemm((int)epi, out.data_ptr(), x.data_ptr(), W.data_ptr(), M, N, K,
                       out.stride(0), ssi, ssn, (float)inv_d, (float)eps, sso, pos, cs, kc, vc, sl,
                       (int)hq, (int)hkv, (int)block_size, cur_stream()),
           "pgemm");
}

void pgemm_variant(int64_t variant, at::Tensor out, at::Tensor x, at::Tensor W) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(W); CHECK_BF16(out);
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && W.size(1) == x.size(1) && out.size(0) == x.size(0) &&
              out.size(1) == W.size(0), "shapes");
  CHECK_RC(omnia_pgemm_variant((int)variant, out.data_ptr(), x.data_ptr(), W.data_ptr(),
                               x.size(0), W.size(0), x.size(1), cur_stream()),
           "pgemm_variant");
}

// split-K 256x256 MFMA GEMM (pgemm.hip EPI 4): parts fp16 [S, M, N] whose sum
// over S is x @ W^T; sched 0 / 1 = 8-wave / 4-wave main loop
void pgemm_splitk(at::Tensor parts, at::Tensor x, at::Tensor W, int64_t sched) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(W);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && W.size(1) == x.size(1), "x [M, K], W [N, K]");
  TORCH_CHECK(x.is_contiguous() && W.is_contiguous(), "contiguous x / W");
  TORCH_CHECK(parts.scalar_type() == at::kHalf && parts.is_contiguous() && parts.dim() == 3 &&
              parts.size(1) == x.size(0) && parts.size(2) == W.size(0), "parts fp16 [S, M, N]");
  TORCH_CHECK(x.device() == W.device() && x.device() == parts.device(), "same device");
  if (x.size(0) == 0) return;
  CHECK_RC(omnia_pgemm_splitk(parts.data_ptr(), x.data_ptr(), W.data_ptr(), x.size(0), W.size(0),
                              x.size(1), parts.size(0), (int)sched, cur_stream()),
           "pgemm_splitk");
}

void row_sumsq(at::Tensor ss, at::Tensor x) {
  CHECK_GPU(x); CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x [M, d] rows contiguous");
  TORCH_CHECK(ss.scalar_type() == at::kFloat && ss.is_contiguous() && ss.numel() == x.size(0) &&
              ss.device() == x.device(), "ss fp32 [M]");
  CHECK_RC(omnia_row_sumsq(ss.data_ptr<float>(), x.data_ptr(), x.size(0), x.size(1), x.stride(0),
                           cur_stream()),
           "row_sumsq");
}

// ------------------------------------------------- split-K consumers (splitk.hip)
// fp32 slabs, or fp16 ones (tgemm mode 3); returns 1 for fp16
static int check_parts(const at::Tensor& p) {
  TORCH_CHECK(p.is_cuda() && (p.scalar_type() == at::kFloat || p.scalar_type() == at::kHalf) &&
              p.is_contiguous() && p.dim() == 3, "parts: contiguous fp32 / fp16 [S, M, N]");
  TORCH_CHECK(p.size(0) >= 1 && p.size(0) <= 16, "1 <= S <= 16");
  return p.scalar_type() == at::kHalf ? 1 : 0;
}

void splitk_add_rmsnorm(at::Tensor out, at::Tensor parts, at::Tensor residual, at::Tensor w,
                        double eps) {
  const int half = check_parts(parts);
  CHECK_BF16(out); CHECK_BF16(residual); CHECK_BF16(w);
  const int M = parts.size(1), d = parts.size(2);
  TORCH_CHECK(residual.is_contiguous() && residual.size(0) == M && residual.size(1) == d,
              "residual [M, d]");
  TORCH_CHECK(out.is_contiguous() && out.size(0) == M && out.size(1) == d, "out [M, d]");
  TORCH_CHECK(w.numel() == d, "w [d]");
  CHECK_RC(omnia_splitk_add_rmsnorm(out.data_ptr(), parts.data_ptr(), half, residual.data_ptr(),
                                    w.data_ptr(), parts.size(0), M, d, (float)eps, cur_stream()),
           "splitk_add_rmsnorm");
}

void splitk_rope_kv(at::Tensor q, at::Tensor parts, at::Tensor positions, at::Tensor cos_sin,
                    at::Tensor k_cache, at::Tensor v_cache, at::Tensor slots, int64_t hq,
                    int64_t hkv, int64_t block_size) {
  const int half = check_parts(parts);
  CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache); CHECK_I32(positions);
  const int T = parts.size(1);
  TORCH_CHECK(parts.size(2) == (hq + 2 * hkv) * 128, "parts N = (hq + 2 hkv) * 128");
  TORCH_CHECK(q.is_contiguous() && q.size(0) == T && q.size(1) == hq * 128, "q [T, hq*128]");
  TORCH_CHECK(positions.numel() == T && slots.numel() == T, "positions / slots [T]");
  TORCH_CHECK(slots.scalar_type() == at::kLong, "slots int64");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == 128, "cos_sin");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == hkv && k_cache.size(2) == block_size &&
              k_cache.size(3) == 128 && k_cache.is_contiguous() && v_cache.is_contiguous(),
              "cache [NB, Hkv, BS, 128]");
  CHECK_RC(omnia_splitk_rope_kv(q.data_ptr(), parts.data_ptr(), half, parts.size(0), T,
                                positions.data_ptr<int>(), cos_sin.data_ptr<float>(),
                                k_cache.data_ptr(), v_cache.data_ptr(),
                                slots.data_ptr<int64_t>(), hq, hkv, 128, block_size,
                                cur_stream()),
           "splitk_rope_kv");
}

void splitk_swiglu(at::Tensor out, at::Tensor parts) {
  const int half = check_parts(parts);
  CHECK_BF16(out);
  const int M = parts.size(1), I = parts.size(2) / 2;
  TORCH_CHECK(parts.size(2) % 2 == 0 && out.is_contiguous() && out.size(0) == M &&
              out.size(1) == I, "out [M, I] for parts [S, M, 2I]");
  CHECK_RC(omnia_splitk_swiglu(out.data_ptr(), parts.data_ptr(), half, parts.size(0), M, I,
                               cur_stream()), "splitk_swiglu");
}

void splitk_reduce(at::Tensor out, at::Tensor parts) {
  const int half = check_parts(parts);
  CHECK_BF16(out);
  TORCH_CHECK(out.is_contiguous() && out.numel() == parts.size(1) * parts.size(2), "out [M, N]");
  CHECK_RC(omnia_splitk_reduce(out.data_ptr(), parts.data_ptr(), half, parts.size(0),
                               out.numel(), cur_stream()), "splitk_reduce");
}

// ------------------------------------------------- one-shot IPC all-reduce (K16)
int64_t ipc_alloc(int64_t bytes) {
  void* p = nullptr;
  CHECK_RC(omnia_ipc_alloc(&p, bytes), "ipc_alloc");
  return reinterpret_cast<int64_t>(p);
}
void ipc_free(int64_t ptr) { CHECK_RC(omnia_ipc_free(reinterpret_cast<void*>(ptr)), "ipc_free"); }
py::bytes ipc_get_handle(int64_t ptr) {
  std::string h(omnia_ipc_handle_size(), '\0');
  CHECK_RC(omnia_ipc_get_handle(reinterpret_cast<void*>(ptr), &h[0]), "ipc_get_handle");
  return py::bytes(h);
}
int64_t ipc_open(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK((int)h.size() == omnia_ipc_handle_size(), "bad IPC handle size");
  void* p = nullptr;
  CHECK_RC(omnia_ipc_open(h.data(), &p), "ipc_open");
  return reinterpret_cast<int64_t>(p);
}
void ipc_close(int64_t ptr) { CHECK_RC(omnia_ipc_close(reinterpret_cast<void*>(ptr)), "ipc_close"); }

// regions: int64 CPU tensor [world] of region base pointers (own + opened peers)
void ar_oneshot(at::Tensor out, at::Tensor in, at::Tensor regions, at::Tensor epochs,
                at::Tensor err, int64_t slot_bytes, int64_t rank) {
  CHECK_GPU(in); CHECK_BF16(in); CHECK_BF16(out); CHECK_I32(epochs); CHECK_I32(err);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel(), "contig");
  TORCH_CHECK(regions.device().is_cpu() && regions.scalar_type() == at::kLong, "regions cpu i64");
  TORCH_CHECK(epochs.numel() >= omnia_ar_blocks(), "epochs per block");
  const int world = regions.numel();
  TORCH_CHECK(world <= omnia_ar_max_ranks(), "world too large");
  std::vector<void*> regs(world);
  for (int p = 0; p < world; ++p) regs[p] = reinterpret_cast<void*>(regions.data_ptr<int64_t>()[p]);
  CHECK_RC(omnia_ar_oneshot(out.data_ptr(), in.data_ptr(), regs.data(), epochs.data_ptr<int>(),
                            err.data_ptr<int>(), in.numel(), slot_bytes, (int)rank, world,
                            cur_stream()), "ar_oneshot");
}

// all-gather of any contiguous tensor's bytes over the IPC regions: out holds
// world x in.nbytes (rank order)
void ar_allgather(at::Tensor out, at::Tensor in, at::Tensor regions, at::Tensor epochs,
                  at::Tensor err, int64_t slot_bytes, int64_t rank) {
  CHECK_GPU(in); CHECK_GPU(out); CHECK_I32(epochs); CHECK_I32(err);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(regions.device().is_cpu() && regions.scalar_type() == at::kLong, "regions cpu i64");
  TORCH_CHECK(epochs.numel() >= omnia_ar_blocks(), "epochs per block");
  const int world = regions.numel();
  TORCH_CHECK(world <= omnia_ar_max_ranks(), "world too large");
  const int64_t nb = in.numel() * in.element_size();
  TORCH_CHECK(out.numel() * out.element_size() == nb * world, "out must hold world x in bytes");
  std::vector<void*> regs(world);
  for (int p = 0; p < world; ++p) regs[p] = reinterpret_cast<void*>(regions.data_ptr<int64_t>()[p]);
  CHECK_RC(omnia_ar_allgather(out.data_ptr(), in.data_ptr(), regs.data(), epochs.data_ptr<int>(),
                              err.data_ptr<int>(), nb, slot_bytes, (int)rank, world,
                              cur_stream()), "ar_allgather");
}

// IPC all-to-all: in / out [world][chunk] (any dtype, chunk bytes % 16 == 0)
void ar_alltoall(at::Tensor out, at::Tensor in, at::Tensor regions, at::Tensor epochs,
                 at::Tensor err, int64_t slot_bytes, int64_t rank) {
  CHECK_GPU(in); CHECK_GPU(out); CHECK_I32(epochs); CHECK_I32(err);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(in.device() == out.device() && epochs.device() == in.device() &&
              err.device() == in.device(), "same device");
  TORCH_CHECK(regions.device().is_cpu() && regions.scalar_type() == at::kLong, "regions cpu i64");
  TORCH_CHECK(epochs.numel() >= omnia_ar_blocks(), "epochs per block");
  const int world = regions.numel();
  TORCH_CHECK(world <= omnia_ar_max_ranks(), "world too large");
  const int64_t nb = in.numel() * in.element_size();
  TORCH_CHECK(out.numel() * out.element_size() == nb && nb % world == 0,
              "in / out: [world][chunk] bytes");
  std::vector<void*> regs(world);
  for (int p = 0; p < world; ++p) regs[p] = reinterpret_cast<void*>(regions.data_ptr<int64_t>()[p]);
  CHECK_RC(omnia_ar_alltoall(out.data_ptr(), in.data_ptr(), regs.data(), epochs.data_ptr<int>(),
                             err.data_ptr<int>(), nb / world, slot_bytes, (int)rank, world,
                             cur_stream()), "ar_alltoall");
}

// IPC point-to-point: out <- rank src's `in` (same bytes on every rank)
void ar_sendrecv(at::Tensor out, at::Tensor in, at::Tensor regions, at::Tensor epochs,
                 at::Tensor err, int64_t slot_bytes, int64_t rank, int64_t src) {
  CHECK_GPU(in); CHECK_GPU(out); CHECK_I32(epochs); CHECK_I32(err);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(in.device() == out.device() && epochs.device() == in.device() &&
              err.device() == in.device(), "same device");
  TORCH_CHECK(regions.device().is_cpu() && regions.scalar_type() == at::kLong, "regions cpu i64");
  TORCH_CHECK(epochs.numel() >= omnia_ar_blocks(), "epochs per block");
  const int world = regions.numel();
  TORCH_CHECK(world <= omnia_ar_max_ranks(), "world too large");
  const int64_t nb = in.numel() * in.element_size();
  TORCH_CHECK(out.numel() * out.element_size() == nb, "out bytes == in bytes");
  std::vector<void*> regs(world);
  for (int p = 0; p < world; ++p) regs[p] = reinterpret_cast<void*>(regions.data_ptr<int64_t>()[p]);
  CHECK_RC(omnia_ar_sendrecv(out.data_ptr(), in.data_ptr(), regs.data(), epochs.data_ptr<int>(),
                             err.data_ptr<int>(), nb, slot_bytes, (int)rank, world, (int)src,
                             cur_stream()), "ar_sendrecv");
}

// two-shot (reduce-scatter + all-gather) over the same IPC regions; with w the
// fused residual add + RMSNorm variant (residual updated in place)
void ar_twoshot(at::Tensor out, at::Tensor in, c10::optional<at::Tensor> residual,
                c10::optional<at::Tensor> w, at::Tensor regions, at::Tensor epochs, at::Tensor err,
                int64_t slot_bytes, int64_t rank, double eps) {
  CHECK_GPU(in); CHECK_BF16(in); CHECK_BF16(out); CHECK_I32(epochs); CHECK_I32(err);
  TORCH_CHECK(in.dim() == 2 && in.is_contiguous() && out.is_contiguous() &&
              out.sizes() == in.sizes(), "in/out contiguous [M, d]");
  TORCH_CHECK(regions.device().is_cpu() && regions.scalar_type() == at::kLong, "regions cpu i64");
  TORCH_CHECK(epochs.numel() >= omnia_ar_blocks(), "epochs per block");
  const bool norm = w.has_value() && w->defined();
  if (norm) {
    TORCH_CHECK(residual.has_value() && residual->defined(), "NORM needs the residual");
    CHECK_BF16((*residual)); CHECK_BF16((*w));
    TORCH_CHECK(residual->sizes() == in.sizes() && residual->is_contiguous(), "residual [M, d]");
    TORCH_CHECK(w->numel() == in.size(1), "w [d]");
  }
  const int world = regions.numel();
  TORCH_CHECK(world <= omnia_ar_max_ranks(), "world too large");
  std::vector<void*> regs(world);
  for (int p = 0; p < world; ++p) regs[p] = reinterpret_cast<void*>(regions.data_ptr<int64_t>()[p]);
  CHECK_RC(omnia_ar_twoshot(out.data_ptr(), in.data_ptr(), opt_ptr<void>(residual),
                            opt_ptr<void>(w), regs.data(), epochs.data_ptr<int>(),
                            err.data_ptr<int>(), in.size(0), in.size(1), slot_bytes, (int)rank,
                            world, (float)eps, cur_stream()), "ar_twoshot");
}

// ------------------------------------------------- host step launch (no GIL churn)
// One decode step = H2D staging copy + graph launch + D2H token copy + event
// record, enqueued back to back on the current stream inside ONE Python call.
// Each separate torch call would drop and re-take the GIL; with a busy asyncio
// serving thread every re-take can wait a full switch interval, starving the
// engine thread and idling the GPU between steps.
void graph_launch_step(int64_t graph_exec, int64_t h2d_dst, int64_t h2d_src, int64_t h2d_bytes,
                       int64_t d2h_dst, int64_t d2h_src, int64_t d2h_bytes, int64_t event) {
  hipStream_t s = cur_stream();
  if (h2d_bytes > 0)
    TORCH_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(h2d_dst),
                               reinterpret_cast<const void*>(h2d_src), h2d_bytes,
                               hipMemcpyHostToDevice, s) == hipSuccess, "H2D staging copy");
  TORCH_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), s) == hipSuccess,
              "hipGraphLaunch");
  if (d2h_bytes > 0)
    TORCH_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(d2h_dst),
                               reinterpret_cast<const void*>(d2h_src), d2h_bytes,
                               hipMemcpyDeviceToHost, s) == hipSuccess, "D2H token copy");
  if (event)
    TORCH_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(event), s) == hipSuccess,
                "hipEventRecord");
}

// Same step, but the staging upload is a compute-queue kernel reading the
// mapped pinned buffer (`src_dev` = omnia_host_device_ptr of it) instead of an
// SDMA copy the compute queue would have to wait on; only the scalar head and
// the [rows x row_bytes] block-table window the graph bucket reads are moved.
void graph_launch_staged(int64_t graph_exec, int64_t dst, int64_t src_dev, int64_t head_bytes,
                         int64_t bt_off, int64_t row_stride, int64_t rows, int64_t row_bytes,
                         int64_t d2h_dst, int64_t d2h_src, int64_t d2h_bytes, int64_t event) {
  hipStream_t s = cur_stream();
  TORCH_CHECK(dst && src_dev && rows >= 0 && rows <= (1 << 20), "bad staging operands");
  CHECK_RC(omnia_stage_copy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src_dev),
                            head_bytes, bt_off, row_stride, (int)rows, row_bytes, s),
           "stage_copy");
  TORCH_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), s) == hipSuccess,
              "hipGraphLaunch");
  if (d2h_bytes > 0)
    TORCH_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(d2h_dst),
                               reinterpret_cast<const void*>(d2h_src), d2h_bytes,
                               hipMemcpyDeviceToHost, s) == hipSuccess, "D2H token copy");
  if (event)
    TORCH_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(event), s) == hipSuccess,
                "hipEventRecord");
}

// standalone staged upload (tests / non-graph paths)
void stage_copy(int64_t dst, int64_t src_dev, int64_t head_bytes, int64_t bt_off,
                int64_t row_stride, int64_t rows, int64_t row_bytes) {
  TORCH_CHECK(dst && src_dev && rows >= 0 && rows <= (1 << 20), "bad staging operands");
  CHECK_RC(omnia_stage_copy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src_dev),
                            head_bytes, bt_off, row_stride, (int)rows, row_bytes, cur_stream()),
           "stage_copy");
}

int64_t host_device_ptr(at::Tensor host) {
  TORCH_CHECK(host.is_pinned(), "host_device_ptr needs a pinned tensor");
  return omnia_host_device_ptr(host.data_ptr());
}

int64_t event_create() {
  hipEvent_t e;
  TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess,
              "hipEventCreate");
  return reinterpret_cast<int64_t>(e);
}

void event_destroy(int64_t e) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e)); }

bool event_query(int64_t e) {
  return hipEventQuery(reinterpret_cast<hipEvent_t>(e)) == hipSuccess;
}

// wait for an event; the GIL is released only if it has not completed yet.
// Returns the nanoseconds spent re-acquiring the GIL after the event fired
// (the serving thread's hold time -- a direct measure of GIL contention).
int64_t event_sync(int64_t e) {
  auto ev = reinterpret_cast<hipEvent_t>(e);
  if (hipEventQuery(ev) == hipSuccess) return 0;
  std::chrono::steady_clock::time_point done;
  {
    py::gil_scoped_release rel;
    TORCH_CHECK(hipEventSynchronize(ev) == hipSuccess, "hipEventSynchronize");
    done = std::chrono::steady_clock::now();
  }
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now() - done).count();
}

}  // namespace

PYBIND11_MODULE(_omnia_kernels, m) {
  m.doc() = "omnia_amd hand-written CDNA4 (gfx950) HIP kernels";
  m.def("rmsnorm", &rmsnorm);
  m.def("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.def("rope_kv", &rope_kv);
  m.def("silu_mul", &silu_mul);
  m.def("embedding", &embedding, py::arg("out"), py::arg("ids"), py::arg("w"),
        py::arg("vocab_start"), py::arg("src") = py::none(), py::arg("tok_slots") = py::none());
  m.def("decode_attention", &decode_attention);
  m.def("prefill_attention", &prefill_attention, py::arg("out"), py::arg("q"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"), py::arg("q_start_loc"),
        py::arg("seq_lens"), py::arg("tile_seq"), py::arg("tile_q0"), py::arg("scale"),
        py::arg("hp") = 0, py::arg("q_tile") = 64, py::arg("lse") = py::none(),
        py::arg("kv_lens") = py::none());
  m.def("sample", &sample, py::arg("out_tok"), py::arg("out_logprob"), py::arg("logits"),
        py::arg("temperature"), py::arg("top_k"), py::arg("top_p"), py::arg("seeds"),
        py::arg("steps"), py::arg("counts"), py::arg("freq_pen"), py::arg("pres_pen"),
        py::arg("rep_pen"), py::arg("tok_slots") = py::none(), py::arg("dst") = py::none());
  m.def("mean_pool_l2", &mean_pool_l2);
  m.def("cosine_scores", &cosine_scores);
  m.def("topk", &topk);
  m.def("moe_topk", &moe_topk);
  m.def("moe_router_topk", &moe_router_topk);
  m.def("moe_max_blocks", &moe_max_blocks, py::arg("n_assign"), py::arg("n_experts"),
        py::arg("bm") = 64);
  m.def("pgemm_moe", &pgemm_moe);
  m.def("moe_align", &moe_align);
  m.def("moe_gemm", &moe_gemm);
  m.def("moe_combine", &moe_combine);
  m.def("dgemm", &dgemm);
  m.def("wgemm", &wgemm);
  m.def("wgemm_wide", &wgemm_wide);
  m.def("tgemm", &tgemm);
  m.def("pgemm", &pgemm);
  m.def("row_sumsq", &row_sumsq);
  m.def("pgemm_variant", &pgemm_variant);
  m.def("pgemm_splitk", &pgemm_splitk);
  m.def("pgemm_set_schedule", [](int64_t sched) {
    TORCH_CHECK(omnia_pgemm_set_schedule((int)sched) == 0, "pgemm schedule must be 0 or 1");
  });
  m.def("ar_twoshot", &ar_twoshot);
  m.def("ar_region_bytes", &omnia_ar_region_bytes);
  m.def("splitk_add_rmsnorm", &splitk_add_rmsnorm);
  m.def("splitk_rope_kv", &splitk_rope_kv);
  m.def("splitk_swiglu", &splitk_swiglu);
  m.def("splitk_reduce", &splitk_reduce);
  m.def("ipc_alloc", &ipc_alloc);
  m.def("ipc_free", &ipc_free);
  m.def("ipc_get_handle", &ipc_get_handle);
  m.def("ipc_open", &ipc_open);
  m.def("ipc_close", &ipc_close);
  m.def("ar_oneshot", &ar_oneshot);
  m.def("ar_allgather", &ar_allgather);
  m.def("ar_alltoall", &ar_alltoall);
  m.def("ar_sendrecv", &ar_sendrecv);
  m.def("ar_blocks", &omnia_ar_blocks);
  m.def("ar_max_ranks", &omnia_ar_max_ranks);
  m.def("apply_token_mask", &apply_token_mask);
  m.def("tp_gumbel", &tp_gumbel);
  m.def("tp_pack", &tp_pack);
  m.def("tp_merge", &tp_merge);
  m.def("graph_launch_step", &graph_launch_step);
  m.def("graph_launch_staged", &graph_launch_staged);
  m.def("stage_copy", &stage_copy);
  m.def("host_device_ptr", &host_device_ptr);
  m.def("event_create", &event_create);
  m.def("event_destroy", &event_destroy);
  m.def("event_query", &event_query);
  m.def("event_sync", &event_sync);
  m.attr("arch") = "gfx950";
}
