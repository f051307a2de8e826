/*
 * yalm_hip.h — the drop-in C ABI of the MI355X (gfx950) decode engine.
 *
 * This header replaces the GPU-facing interface of the reference
 * (/root/reference/src/model.h:33-39, 70-79, 353-385 and the C++ members
 * compiled in src/infer.cu). It contains no HIP, CUDA or C++ types: every
 * entry point takes plain pointers, sizes and POD structs, so the reference's
 * own host (model.cpp, main.cpp, test.cpp) — or our C++20 mirror of it under
 * yalm_amd/host/ — binds it directly.
 *
 * Errors: every int-returning function returns YALM_OK (0) or a YALM_ERR_*
 * code; yalm_last_error() describes the last failure on the calling thread.
 * (The reference aborts on any runtime error, infer.cu:13-31; callers that
 * want that behaviour check the code and abort.)
 *
 * Threading: one decoder per stream; a decoder is not re-entrant (same as the
 * reference's InferenceState, model.h:84-190).
 */
#ifndef YALM_HIP_H
#define YALM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YALM_OK 0
#define YALM_ERR_HIP 1         /* a HIP runtime call failed */
#define YALM_ERR_ARG 2         /* bad argument / shape */
#define YALM_ERR_UNSUPPORTED 3 /* configuration the kernels do not implement */

/* DType codes follow the reference enum order (codec.h:15-25). */
enum { YALM_F32 = 0, YALM_F16 = 1, YALM_BF16 = 2, YALM_F8E5M2 = 3 };
/* ActivationType (model.h:14-17) */
enum { YALM_GELU = 0, YALM_SILU = 1 };
/* InferenceMode (model.h:28-31) */
enum { YALM_HYDRATE_KV_CACHE = 0, YALM_OUTPUT_LOGITS = 1 };

/* Opaque stream handle; replaces cudaStream_t in init_cuda_stream (model.h:39). */
typedef struct yalm_stream_s *yalm_stream;
/* Opaque decoder: the device half of InferenceState + Model (model.h:84-190,
 * 303-327) — scratch buffers, KV caches, per-mode hipGraphs. */
typedef struct yalm_decoder_s *yalm_decoder;

/* Config (model.h:41-68). Same field meaning; MoE fields are not carried
 * because the reference GPU path asserts on MoE (infer.cu:865-867). */
typedef struct yalm_config {
	int dim, hidden_dim, head_dim, n_layers, n_heads, n_kv_heads, vocab_size, max_seq_len;
	float rope_theta;
	int rotary_dim;
	float norm_eps;
	int act;          /* YALM_GELU / YALM_SILU */
	float qkv_clip;   /* FLT_MAX when absent (model.cpp:60-61) */
	int weight_dtype; /* YALM_F32 / YALM_F16 / YALM_F8E5M2 */
} yalm_config;

/* Device pointers of one block (Block private fields, model.h:286-300). If
 * key_cache/value_cache are NULL the decoder allocates them (zeroed,
 * max_seq_len x n_kv_heads x head_dim f16 each). */
typedef struct yalm_block_weights {
	const float *rms_att, *rms_ffn;
	const void *wq, *wk, *wv, *wo, *w1, *w2, *w3;
	uint16_t *key_cache, *value_cache;
} yalm_block_weights;

/* Device pointers of the model (Model fields, model.h:303-311). wcls may equal
 * token_embedding (tied weights, model.cpp:370-377). blocks is a HOST array
 * of n_layers entries, copied by yalm_decoder_create. */
typedef struct yalm_model_weights {
	const void *token_embedding;
	const float *rms_final;
	const void *wcls;
	const yalm_block_weights *blocks;
} yalm_model_weights;

/* ---------------- device shim: replaces model.h:33-39 / infer.cu:59-90 ---------------- */
const char *yalm_last_error(void);
/* set_cuda_device (model.h:38): selects the HIP device for this thread. */
int yalm_set_device(int device);
/* upload_cuda (model.h:33): device alloc + H2D copy; returns NULL on failure. */
void *yalm_upload(const void *host, size_t size);
/* device alloc (zero-filled); returns NULL on failure. */
void *yalm_alloc(size_t size);
/* download_cuda (model.h:34): D2H copy into a caller buffer (the reference
 * allocated pinned memory and passed std::string through extern "C"). */
int yalm_download(void *host, const void *device, size_t size);
/* register_cuda_host / unregister_cuda_host (model.h:35, 37). */
int yalm_register_host(void *host, size_t size);
int yalm_unregister_host(void *host);
/* free_cuda (model.h:36). */
int yalm_free(void *device);
/* init_cuda_stream (model.h:39), with an opaque handle. */
int yalm_stream_create(yalm_stream *out);
int yalm_stream_destroy(yalm_stream s);
int yalm_stream_sync(yalm_stream s);
/* Fill n device elements of dtype with the deterministic synthetic
 * initialiser (uniform in [offset-scale, offset+scale); f32 adds offset).
 * Used to build random-weight models of real shapes in HBM without a PCIe
 * upload (bench.py). Same integer hash as the CPU oracle. */
int yalm_synth(void *device, size_t n, int dtype, uint64_t seed, float scale, float offset, yalm_stream s);

/* ---------------- decoder: replaces Model::_forward_cuda / Block::_block_cuda ---------------- */
/* Creates the device state for one sequence (InferenceState::cuda,
 * model.cpp:323-345) on stream s (NULL = a private stream). Weight pointers
 * must stay valid for the decoder's lifetime. */
int yalm_decoder_create(const yalm_config *config, const yalm_model_weights *weights, yalm_stream s,
                        yalm_decoder *out);
int yalm_decoder_destroy(yalm_decoder d);
/* Model::forward (model.cpp:396-407 -> infer.cu:1021-1039): one token through
 * every block at position pos (sliding-window/sink indices as infer.cu:1081-
 * 1083). mode YALM_OUTPUT_LOGITS also computes the final norm + logits and,
 * if logits_host != NULL, copies vocab_size floats there before returning
 * (synchronous, like the reference's OUTPUT mode). YALM_HYDRATE_KV_CACHE is
 * asynchronous. Graph-replayed after the first call per mode. */
int yalm_forward(yalm_decoder d, int token, int pos, int mode, float *logits_host);
/* Device-resident greedy decode (-t 0; sampler.cpp:27-38 first-max argmax on
 * the device): feeds `token` at `pos`, then n_steps-1 more tokens each chosen
 * by argmax of the previous step; writes the n_steps argmax tokens to
 * out_tokens (host). No host round trip per token: each token's kernels are
 * launched back to back (eagerly: measured 0.3-0.5% faster than replaying the
 * per-token graph, whose kernel count yalm_graph_kernels still reports). */
int yalm_generate_greedy(yalm_decoder d, int token, int pos, int n_steps, int *out_tokens);
/* Launch-only variant for benchmarking: enqueue n_steps greedy steps
 * continuing from the decoder's device-resident token/pos; no sync. */
int yalm_enqueue_greedy(yalm_decoder d, int n_steps);
/* Read back the device-resident next token / position after enqueue+sync. */
int yalm_device_step(yalm_decoder d, int *token, int *pos);
/* The greedy tokens produced on the device since the last yalm_generate_greedy
 * (that call's tokens, then every yalm_enqueue_greedy step, up to 65536):
 * copies min(*n_total, cap) of them to out (host) after a sync; *n_total = how many
 * were produced. Lets tensor-parallel ranks compare whole sequences (bench.py). */
int yalm_device_tokens(yalm_decoder d, int *out, int cap, int *n_total);
/* Block::block (model.cpp:213-265) for one layer, eagerly, on the decoder's
 * current activation x (the test hook for per-layer parity). */
int yalm_block(yalm_decoder d, int layer, int pos, int kv_sink, int kv_pos, int kv_len);
/* Host access to the decoder's activation x (dim floats) and logits. After a
 * YALM_HYDRATE_KV_CACHE forward of an IPC tensor-parallel decoder x is undefined
 * (that forward's last W2 partial is never exchanged: nothing reads it); after
 * yalm_block and OUTPUT forwards it is the full hidden state on every rank. */
int yalm_get_x(yalm_decoder d, float *host);
int yalm_set_x(yalm_decoder d, const float *host);
int yalm_get_logits(yalm_decoder d, float *host);
/* Average device time (ms) of one kernel of the forward, launched eagerly on
 * the decoder's stream `iters` times between HIP events (layers rotated so the
 * weights come from HBM). kernel_id: 0 = QKV GEMV, 1 = attention, 2 = Wo GEMV,
 * 3 = W1/W3 GEMV+GLU, 4 = W2 GEMV, 5 = logits GEMV, 6 = one tensor-parallel
 * exchange of x (RCCL all-reduce or IPC exchange; collective: every rank calls it
 * with the same iters), 8 = the fused attention + Wo
 * launch (yalm_decoder_attn_wo; each timed launch gets a fresh step epoch, so its
 * Wo waves wait for the heads as in a real forward; the epoch-bump launches are
 * timed separately and subtracted). Used by bench.py for the roofline of the
 * dominant kernel. */
int yalm_time_kernel(yalm_decoder d, int kernel_id, int iters, float *avg_ms);
/* The same-process streaming envelope: average ms of one pure read-only pass over
 * `bytes` of HBM (16-byte non-temporal loads, the best of a few wave geometries,
 * `iters` back-to-back launches alternating two buffers so the 256 MiB Infinity
 * Cache cannot serve them). bench.py reports a kernel's time against it so the
 * roofline fraction is also stated relative to what THIS box streams. */
int yalm_stream_envelope(size_t bytes, int iters, float *avg_ms);
/* Override the GEMV launch geometry of one weight-streaming kernel kind
 * (0 = QKV, 1 = Wo, 2 = W1/W3, 3 = W2, 4 = logits): workgroup size
 * 256|512|1024, unroll (16-byte loads in flight per lane) 2|4|8, and `gpw` =
 * workgroups per CU of the row-block kernel; 0 = automatic.
 * Drops captured graphs (re-captured on next use). Tuning/ablation hook. */
int yalm_set_gemv_config(yalm_decoder d, int kind, int threads, int unroll, int gpw);
/* Kernel launches per forward of graph `mode` (0 = HYDRATE, 1 = OUTPUT_LOGITS, 2 = the
 * device greedy step): *kernels = kernel nodes of the captured per-token hipGraph (RCCL
 * collectives count as the kernels they capture), *nodes (may be NULL) = all nodes. Test
 * and measurement hook (tensor parallelism adds no exchange launches over IPC). */
int yalm_graph_kernels(yalm_decoder d, int mode, int *kernels, int *nodes);
/* Name of kernel_id's device function (to match rocprofv3 summaries). */
const char *yalm_kernel_name(yalm_decoder d, int kernel_id);
/* 1 if this decoder's launch path runs attention and the Wo projection (+ the
 * residual add) as ONE launch (attn_wo.h: the Wo weight stream overlaps the
 * attention; replaces attn + fused_matmul_add_residuals, infer.cu:338-524, 270):
 * head_dim 128, fp16 / fp8 weights with 1, 2, 4 or 8 KB (per-rank) Wo rows, and
 * not YALM_LAUNCH_SEPARATE_ATTN_WO. 0 = two separate launches. The split-KV
 * attention output is handed to the Wo workgroups as {value, epoch} granules. */
int yalm_decoder_attn_wo(yalm_decoder d);
/* Launch-mode switches of one decoder (default 0; drops captured graphs):
 * YALM_LAUNCH_EAGER every forward launches its kernels directly instead of replaying
 * the per-token graph (profilers that mis-handle graph replay); YALM_LAUNCH_SYNC a
 * stream sync after every replay (debugging); YALM_LAUNCH_SEPARATE_ATTN_WO separate
 * attention and Wo launches where the fused one would run (A/B and tests). The
 * production library reads no environment variable. */
#define YALM_LAUNCH_EAGER 1
#define YALM_LAUNCH_SYNC 2
#define YALM_LAUNCH_SEPARATE_ATTN_WO 4
int yalm_decoder_set_launch(yalm_decoder d, int flags);
/* The fused launch's plan for a (per-rank) config when `slots` workgroups of 256
 * threads are co-resident (occupancy x CUs): returns 1 and the key splits per kv head
 * and the grid size, or 0 = separate attention and Wo launches (unsupported shape, or
 * fewer than 2 key splits fit beside the mergers and Wo workgroups while contexts can
 * exceed head mode). Pure host arithmetic: no device is touched. */
int yalm_attn_wo_plan(const yalm_config *config, int slots, int *splits, int *grid);
/* Timeline of the most recent fused attention + Wo launch (decoder created with
 * YALM_ATTN_WO_TRACE=1): 16 stamps per workgroup at [w * 16 + k]: k < 8
 * s_memrealtime (100 MHz), k + 8 the shader clock (s_memtime) at the same point (k = 0: instead the
 * workgroup's place, HW_ID | XCC_ID << 32); k = 0 start, 1 hand-off signalled (attention; 0 if this workgroup did not
 * finish a kv head) or Wo slice landed (Wo; the trace waits for it), 2 poll passed (Wo) or
 * first K/V/q loads landed (attention; the trace waits for them), 3 end; attention units:
 * 4 scores of the last chunk, 5 its softmax, 6 P.V sums combined, 7 head outputs / partials
 * issued; merger workgroups (2 and 4 read 0): 5 gather issued, 7 every partial seen. A
 * phase a workgroup never reached reads 0. Workgroups [0, *attention_workgroups) are
 * attention units and mergers, the rest Wo. */
int yalm_attn_wo_trace(yalm_decoder d, unsigned long long *host, size_t count, int *workgroups,
                       int *attention_workgroups);

/* ---------------- tensor parallelism (BASELINE config 5) ----------------
 * Megatron row/column split of one model over tp_size GPUs, one process per
 * GPU: rank r holds Wq/Wk/Wv rows of heads [r*H/N, (r+1)*H/N) (kv heads
 * likewise), Wo columns of those heads, W1/W3 rows and W2 columns
 * [r*hidden/N, (r+1)*hidden/N), Wcls rows [r*vocab/N, ..); norms and the
 * embedding are replicated. Each layer then needs two all-reduces of x
 * (after Wo and after W2), captured in the per-token graph as RCCL
 * ncclAllReduce over xGMI; the greedy argmax gathers one (value, index) pair
 * per rank. Replaces the single-device forward of model.cpp:396-407 /
 * infer.cu:1021-1128 for multi-GPU; the reference has no multi-GPU path. */
/* 128-byte RCCL unique id, created by rank 0 and shared with the other ranks
 * out of band (bench.py: torch.distributed broadcast). */
int yalm_tp_unique_id(void *id_out);
/* config: the FULL model; weights: this rank's shards as above (blocks as in
 * yalm_decoder_create, KV caches for the local kv heads or null). Collective:
 * every rank calls it concurrently (ncclCommInitRank). All yalm_forward /
 * yalm_generate_greedy calls must then be made by every rank in lockstep;
 * logits (full vocabulary) and greedy tokens are identical on all ranks. */
int yalm_decoder_create_tp(const yalm_config *config, const yalm_model_weights *weights, int tp_rank, int tp_size,
                           const void *unique_id, yalm_stream s, yalm_decoder *out);
/* The same split with an IPC one-shot exchange instead of RCCL (no NCCL
 * communicator; also runs several ranks on ONE GPU, which RCCL refuses): each
 * rank allocates its exchange buffer (yalm_tp_ipc_alloc, config = full model,
 * s = the stream its decoder will run on) and shares the YALM_TP_HANDLE_BYTES
 * rank record out of band (the buffer's hipIpcMemHandle, the GPU's UUID and the
 * stream's CU mask); every rank then passes all tp_size records (rank order)
 * and the same stream s. Ranks on one GPU whose CU masks overlap get a one-wave
 * gate launch before each exchange consumer (they could otherwise hold the CUs a
 * peer's producer needs); one GPU per rank, or disjoint CU masks
 * (yalm_stream_create_cu_part), run the production sequence without it. The
 * decoder takes ownership of own_buf (1..8 ranks). Per exchange no launch of its own:
 * the producer (the fused attention + Wo launch, the W2 GEMV, the logits GEMV,
 * the argmax) pushes each value of this rank's partial into this rank's slot of
 * EVERY rank's buffer as an 8-byte {value, tag} granule (one system-scope store:
 * the data is its own ready flag); the consumer (the next normalising GEMV)
 * waits for every rank's granules while its weight stream starts and sums them
 * in rank order, so x is identical on every rank. Past 4 ranks a collect launch
 * sums x once before the consumer. The exchange sequence numbers live in the
 * decoder's step state, so every rank must make the same calls in lockstep. */
#define YALM_TP_HANDLE_BYTES 128
#define YALM_CU_MASK_WORDS 8 /* 256 CUs */
int yalm_tp_ipc_alloc(const yalm_config *config, int tp_size, yalm_stream s, void **buf, void *handle_out);
/* A stream restricted to CU block `part` of `n_parts` (CUs [part * ncu / n_parts,
 * (part + 1) * ncu / n_parts), spread by the driver over all XCDs): n_parts rank
 * processes on ONE GPU then run on disjoint CUs like n_parts small GPUs (the
 * one-GPU rehearsal of tensor parallelism; tests/test_gpu_mistral_dims.py, bench.py
 * --rehearse). Destroy with yalm_stream_destroy. */
int yalm_stream_create_cu_part(int part, int n_parts, yalm_stream *out);
int yalm_decoder_create_tp_ipc(const yalm_config *config, const yalm_model_weights *weights, int tp_rank, int tp_size,
                               void *own_buf, const void *handles, yalm_stream s, yalm_decoder *out);
/* Device-to-device 2D copy (hipMemcpy2D): shard slicing of weights resident in HBM. */
int yalm_copy_2d(void *dst, size_t dst_pitch, const void *src, size_t src_pitch, size_t width, size_t height);

/* ---------------- batched prefill (MFMA): the perplexity / prompt path ----------------
 * Replaces the reference's position-by-position forward loop over a prompt
 * (main.cpp:128-200 `-m perplexity`, main.cpp:95-101 prompt hydration,
 * Model::forward per position, model.cpp:396-407) with one pass per layer
 * over all n positions: rmsnorm + QKV GEMM + RoPE + fp16 KV-cache write, causal
 * GQA attention, Wo / W1|W3 / W2 GEMMs on the f16 MFMA units.
 * Fills the KV cache rows pos0 .. pos0 + n - 1 exactly where the decoder
 * expects them, so yalm_forward / yalm_generate_greedy can continue at
 * pos0 + n. logprobs (host, n floats, may be NULL): logprobs[i] =
 * log softmax(logits at position pos0 + i)[tokens[i + 1]] for i < n - 1 (the
 * quantity main.cpp:155 sums), logprobs[n - 1] = 0. Requires f16 weights,
 * dims multiple of 128, head_dim 64 | 128 and pos0 + n <= max_seq_len
 * (the sliding window past max_seq_len stays on the decode path).
 * Synchronous. Activations are rounded to f16 for the MFMA inputs: results
 * match the decode path within the tolerance stated in tests/test_gpu_prefill.py.
 * Range guard: where the reference's f32 activations would not fit an f16 operand,
 * a layer's GLU output (W2's A operand; trained checkpoints' "massive activations")
 * is stored with an exact power-of-two scale that W2's epilogue undoes, and the pass
 * runs again; any other operand out of range (the normalised x, Q) returns
 * YALM_ERR_UNSUPPORTED (the decode path keeps them in f32). */
int yalm_prefill(yalm_decoder d, const int *tokens, int n, int pos0, float *logprobs);
/* The last yalm_prefill's passes (1 = no operand out of range) and the number of
 * layers whose GLU output ran scaled. */
int yalm_prefill_info(yalm_decoder d, int *passes, int *scaled_layers);
/* Precision form of decoder d's prefill. YALM_PREFILL_FAST (default): f16 activation
 * operands (the K / V columns' over a split [hi | lo] operand). YALM_PREFILL_SPLIT: every
 * activation operand -- the normalised x, Q, the attention probabilities P, the attention
 * output, the GLU output -- as f16 [hi | lo] pairs (~22 significant bits, the f32 the
 * reference keeps, to ~2^-22), at twice the matrix work; the perplexity bar of SURVEY §7
 * (|d log ppl| <= 1e-3) then holds on peaked models too. The CLI's
 * -m perplexity uses SPLIT, prompt hydration FAST. */
#define YALM_PREFILL_FAST 0
#define YALM_PREFILL_SPLIT 1
int yalm_set_prefill_precision(yalm_decoder d, int mode);
/* Average device time (ms) of one n-position prefill with log-probs (synthetic
 * token ids), over `iters` back-to-back runs (bench_prefill.py). */
int yalm_prefill_time(yalm_decoder d, int n, int iters, float *avg_ms);
/* Test / ablation hook: the prefill GEMM forms of decoder d (d = NULL: of the
 * yalm_gemm_f16 test hook). spec = comma-separated key:value pairs, NULL or "" = the
 * defaults: qkv|wo|glu|w2|cls|test:<128|192|256|320> force that GEMM's tile width;
 * 8p:0 the 2-phase kernel; persist:0 one workgroup per tile; skinny:0 the large tiles
 * for T <= 64 too; qkv1:0 the q and k|v GEMMs as two launches; skl:0 the skinny GEMMs'
 * weights as register loads; wnorm:0 the row norms as one workgroup per row (default:
 * one wave per row). Every GEMM form is exact against the others (tests). An
 * unknown key is YALM_ERR_ARG. */
int yalm_set_prefill_forms(yalm_decoder d, const char *spec);

/* ---------------- test API: replaces infer.cu:890-1019 (model.h:370-384) ---------------- */
/* Host pointers in and out; synchronous. dtype selects the weight type
 * (matmul_cuda<float|half|uint8_t>). */
int yalm_matmul(float *xout, const float *x, const void *w, int n, int d, int dtype);
/* mha_cuda: xout (n_heads, head_dim), att (n_heads, max_seq_len) softmax
 * probabilities for t < kv_len. */
int yalm_mha(float *xout, float *att, const uint16_t *kb, const uint16_t *vb, const float *q, int head_dim, int kv_len,
             int max_seq_len, int n_heads, int n_kv_heads);
/* ffn_cuda: xout = W2 (act(W1 x) * W3 x). */
int yalm_ffn(float *xout, const float *x, const void *w1, const void *w2, const void *w3, int hidden_dim, int dim,
             int act, int dtype);

/* Device greedy sampling (sampler.cpp:27-38 sample_argmax: strict '>' scan, the
 * FIRST maximum wins, 0 when nothing exceeds -FLT_MAX): *out = argmax of n host
 * logits through argmax_kernel, the kernel of the -t 0 decode loop. n_shards > 1
 * runs the tensor-parallel form instead: one per-shard first max as a (value,
 * global index) pair over each n / n_shards slice, then argmax_pick_kernel. */
int yalm_argmax(const float *logits, int n, int n_shards, int *out);

/* Prefill building blocks (host pointers, synchronous):
 * c[M][N] f32 = a[M][K] f16 · w[N][K]^T f16 (the MFMA GEMM; N % 128 == 0, K % 64 == 0). */
int yalm_gemm_f16(float *c, const uint16_t *a, const uint16_t *w, int M, int N, int K);
/* Causal GQA attention of T query rows at positions pos0 .. pos0 + T - 1:
 * q [T][n_heads * head_dim] f16, kc / vc [pos0 + T][n_kv_heads * head_dim] f16,
 * o [T][n_heads * head_dim] f16 (infer.cpp:216-248 per row and head). */
int yalm_attn_prefill(uint16_t *o, const uint16_t *q, const uint16_t *kc, const uint16_t *vc, int T, int pos0,
                      int n_heads, int n_kv_heads, int head_dim);

#ifdef __cplusplus
}
#endif
#endif
