/*
 * yalm_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * This is a plain-C restatement of the reference's CPU forward pass
 * (/root/reference/src/infer.cpp:48-523, model.cpp:17-75) used ONLY as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg. Nothing in the product (yalm_amd/, include/yalm_hip.h)
 * links, loads or calls it; the product fails loudly without its HIP library.
 *
 * Pinning status: the reference's own CPU kernels are
 * compiled here from /root/reference/src/infer.cpp unmodified (oracle/Makefile
 * `ref-infer`: the genuine cuda_runtime_api.h that ships with triton satisfies
 * model.h) and this restatement's orc_matmul_f32 / orc_matmul_f16 / orc_mha /
 * orc_attn / orc_ffn are BIT-EXACT against their matmul_cpu / mha_cpu / ffn_cpu
 * on the committed outputs (tests/test_ref_infer.py). The per-block glue
 * (_block_cpu's rmsnorm, RoPE, clip, KV write, sink rotation, residual adds) and
 * _forward_cpu need Block / Model objects from model.cpp, which needs spdlog
 * (absent): restated statement by statement, cross-checked against an
 * independent float64 numpy forward in tests/. Also pinned: the reference's
 * known-answer test (test.cpp:68-126) and .yalm fixtures from its convert.py.
 *
 * Arithmetic follows the reference source statement by statement and is
 * compiled with the reference's flags (Makefile:36-39: -O3 -ffast-math -mavx2
 * -mfma -mf16c -fopenmp) so the f16 GEMV summation order (two 8-wide FMA
 * accumulators, infer.cpp:63-98) is reproduced exactly.
 */
#ifndef YALM_ORACLE_H
#define YALM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field meaning as reference Config (model.h:41-68). Layout is identical
 * to yalm_config in include/yalm_hip.h so tests can share one ctypes struct. */
typedef struct orc_config {
	int dim, hidden_dim, head_dim, n_layers, n_heads, n_kv_heads, vocab_size, max_seq_len;
	float rope_theta;
	int rotary_dim;
	float norm_eps;
	int act;          /* 0 = GELU, 1 = SILU (model.h:14-17) */
	float qkv_clip;
	int weight_dtype; /* 0 = F32, 1 = F16, 3 = F8E5M2 (codec.h:15-25 order) */
} orc_config;

/* Block weights on the host (model.h:286-300). */
typedef struct orc_block {
	const float *rms_att, *rms_ffn;
	const void *wq, *wk, *wv, *wo, *w1, *w2, *w3;
	uint16_t *key_cache, *value_cache; /* (max_seq_len, n_kv_heads*head_dim) f16 */
} orc_block;

typedef struct orc_model {
	orc_config c;
	const void *emb;       /* (vocab, dim) */
	const float *rms_final;
	const void *wcls;      /* (vocab, dim), may alias emb */
	const orc_block *blocks;
} orc_model;

/* InferenceState buffers (model.h:168-186). */
typedef struct orc_state {
	float *x, *xb, *xb2, *hb, *hb2, *q, *k, *v, *att, *logits;
} orc_state;

/* infer.cpp:48-98 (+ fp8: E5M2 byte upcast to f16 exactly, then the f16 order) */
void orc_matmul_f32(float *xout, const float *x, const float *w, int n, int d);
void orc_matmul_f16(float *xout, const float *x, const uint16_t *w, int n, int d);
void orc_matmul_f8(float *xout, const float *x, const uint8_t *w, int n, int d);
void orc_rmsnorm(float *o, const float *x, const float *w, int size, float eps);        /* infer.cpp:134-144 */
void orc_rope(float *vec, int d, int head_dim, int pos, float theta, int rotary_dim);    /* infer.cpp:200-213 */
void orc_softmax(float *o, const float *x, int size);                                    /* infer.cpp:170-185 */
void orc_attn(float *xout, float *atth, const float *qh, const uint16_t *kh, const uint16_t *vh, int head_dim,
              int n_kv_heads, int kv_len);                                                 /* infer.cpp:216-248 */
void orc_mha(float *xout, float *att, const uint16_t *kb, const uint16_t *vb, const float *q, int head_dim, int kv_len,
             int max_seq_len, int n_heads, int n_kv_heads);                               /* infer.cpp:387-403 */
void orc_ffn(float *xout, const float *x, const void *w1, const void *w2, const void *w3, int hidden_dim, int dim,
             int act, int weight_dtype);                                                  /* infer.cpp:412-438 */
void orc_block_forward(const orc_config *c, const orc_block *b, orc_state *s, int pos, int kv_sink, int kv_pos,
                       int kv_len);                                                        /* infer.cpp:254-385 */
void orc_forward(const orc_model *m, orc_state *s, int token, int pos, int mode);          /* infer.cpp:474-523 */
void orc_kv_indices(int max_seq_len, int pos, int *kv_sink, int *kv_pos, int *kv_len);   /* infer.cpp:483-485 */
int orc_sample_argmax(const float *logits, int vocab_size);                                /* sampler.cpp:27-38 */
float orc_sample_prob(const float *logits, int vocab_size, int index);                     /* sampler.cpp:11-25 */
void orc_srand(unsigned seed);                                                             /* sampler.cpp:6-9 */
int orc_sample(const float *logits, int vocab_size, float temperature);                    /* sampler.cpp:40-65 */

/* Deterministic synthetic weights (same integer hash as the product's device
 * initialiser; used to reproduce the bench's random-weight model on the host). */
void orc_synth_f32(float *dst, size_t n, uint64_t seed, float scale, float offset);
void orc_synth_f16(uint16_t *dst, size_t n, uint64_t seed, float scale);
void orc_synth_f8(uint8_t *dst, size_t n, uint64_t seed, float scale);
void orc_set_threads(int n);
int orc_get_threads(void);

#ifdef __cplusplus
}
#endif
#endif
