/*
 * yalm_oracle.c — CPU ORACLE (test infrastructure only; see yalm_oracle.h).
 *
 * Plain-C restatement of /root/reference/src/infer.cpp. Each function cites
 * the reference lines it follows. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this library (as liboracle.so).
 */
#include "yalm_oracle.h"

#include <assert.h>
#include <float.h>
#include <immintrin.h>
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

/* infer.cpp:11-16 */
static inline float half_to_float(uint16_t x) {
	return _cvtsh_ss(x);
}
static inline uint16_t float_to_half(float x) {
	return _cvtss_sh(x, 0);
}

/* infer.cpp:48-59 */
void orc_matmul_f32(float *xout, const float *x, const float *w, int n, int d) {
	int i;
#pragma omp parallel for private(i)
	for (i = 0; i < d; i++) {
		float val = 0.0f;
		for (int j = 0; j < n; j++) {
			val += w[(size_t)i * n + j] * x[j];
		}
		xout[i] = val;
	}
}

/* infer.cpp:63-98: two 8-wide FMA accumulators over 16-element chunks, then
 * sum8 = lo + hi, sum4 = sum8[0:4] + sum8[4:8], dp_ps(sum4, 1, 0xf1). */
static inline float reduce_lohi(__m256 sumlo, __m256 sumhi) {
	__m256 sum8 = _mm256_add_ps(sumlo, sumhi);
	__m128 sum4 = _mm_add_ps(_mm256_extractf128_ps(sum8, 0), _mm256_extractf128_ps(sum8, 1));
	__m128 sum1 = _mm_dp_ps(sum4, _mm_set1_ps(1.0f), 0xf1);
	return _mm_cvtss_f32(sum1);
}

void orc_matmul_f16(float *xout, const float *x, const uint16_t *w, int n, int d) {
	assert(n % 16 == 0);
	int i;
#pragma omp parallel for private(i)
	for (i = 0; i < d; i++) {
		__m256 sumlo = _mm256_setzero_ps();
		__m256 sumhi = _mm256_setzero_ps();
		const uint16_t *row = w + (size_t)i * n;
		for (int j = 0; j < n; j += 16) {
			__m256i wvec = _mm256_loadu_si256((const __m256i *)&row[j]);
			__m128i wveclo = _mm256_extractf128_si256(wvec, 0);
			__m128i wvechi = _mm256_extractf128_si256(wvec, 1);
			__m256 wveclo_ps = _mm256_cvtph_ps(wveclo);
			__m256 wvechi_ps = _mm256_cvtph_ps(wvechi);
			__m256 xveclo = _mm256_loadu_ps(&x[j]);
			__m256 xvechi = _mm256_loadu_ps(&x[j + 8]);
			sumlo = _mm256_fmadd_ps(wveclo_ps, xveclo, sumlo);
			sumhi = _mm256_fmadd_ps(wvechi_ps, xvechi, sumhi);
		}
		xout[i] = reduce_lohi(sumlo, sumhi);
	}
}

/* fp8 E5M2 weights. The reference reads these bytes as f16 (infer.cpp:460-467,
 * 515-518: out of bounds), so the reference defines no fp8 result.
 * Defined here as: every E5M2 byte b is the f16 value with bits (b << 8) — an
 * exact upcast — followed by exactly the f16 GEMV order above. This equals the
 * reference f16 path run on an "fp16 twin" of the file. */
void orc_matmul_f8(float *xout, const float *x, const uint8_t *w, int n, int d) {
	assert(n % 16 == 0);
	int i;
	const __m128i zero = _mm_setzero_si128();
#pragma omp parallel for private(i)
	for (i = 0; i < d; i++) {
		__m256 sumlo = _mm256_setzero_ps();
		__m256 sumhi = _mm256_setzero_ps();
		const uint8_t *row = w + (size_t)i * n;
		for (int j = 0; j < n; j += 16) {
			__m128i b = _mm_loadu_si128((const __m128i *)&row[j]);
			__m128i wveclo = _mm_unpacklo_epi8(zero, b); /* f16 bits = byte << 8 */
			__m128i wvechi = _mm_unpackhi_epi8(zero, b);
			__m256 wveclo_ps = _mm256_cvtph_ps(wveclo);
			__m256 wvechi_ps = _mm256_cvtph_ps(wvechi);
			__m256 xveclo = _mm256_loadu_ps(&x[j]);
			__m256 xvechi = _mm256_loadu_ps(&x[j + 8]);
			sumlo = _mm256_fmadd_ps(wveclo_ps, xveclo, sumlo);
			sumhi = _mm256_fmadd_ps(wvechi_ps, xvechi, sumhi);
		}
		xout[i] = reduce_lohi(sumlo, sumhi);
	}
}

static void matmul_any(float *xout, const float *x, const void *w, int n, int d, int dtype) {
	switch (dtype) {
	case 0:
		orc_matmul_f32(xout, x, (const float *)w, n, d);
		break;
	case 1:
		orc_matmul_f16(xout, x, (const uint16_t *)w, n, d);
		break;
	case 3:
		orc_matmul_f8(xout, x, (const uint8_t *)w, n, d);
		break;
	default:
		abort();
	}
}

static size_t dtype_size(int dtype) {
	return dtype == 0 ? 4 : dtype == 1 ? 2 : 1;
}

/* infer.cpp:134-144 */
void orc_rmsnorm(float *o, const float *x, const float *weight, int size, float eps) {
	float rms = 0.0f;
	for (int i = 0; i < size; ++i) {
		rms += x[i] * x[i];
	}
	rms = sqrtf(rms / size + eps);
	float scale = 1.0f / rms;
	for (int i = 0; i < size; ++i) {
		o[i] = x[i] * scale * weight[i];
	}
}

/* infer.cpp:170-185 */
static void softmax(float *o, const float *x, int size) {
	float score_max = -FLT_MAX;
	for (int i = 0; i < size; ++i) {
		if (x[i] > score_max) {
			score_max = x[i];
		}
	}
	float score_sum = 0.0f;
	for (int i = 0; i < size; ++i) {
		o[i] = expf(x[i] - score_max);
		score_sum += o[i];
	}
	for (int i = 0; i < size; ++i) {
		o[i] /= score_sum;
	}
}

void orc_softmax(float *o, const float *x, int size) {
	softmax(o, x, size);
}

/* infer.cpp:187-197 */
static inline float gelu(float x) {
	return 0.5f * x * (1.0f + tanhf(0.797885f * (x + 0.044715f * x * x * x)));
}
static inline float silu(float x) {
	return x / (1.0f + expf(-x));
}
static inline float clip(float x, float v) {
	return x < -v ? -v : (x > v ? v : x);
}

/* infer.cpp:200-213: interleaved-pair RoPE */
void orc_rope(float *vec, int d, int head_dim, int pos, float theta, int rotary_dim) {
	for (int i = 0; i < d; i += 2) {
		int j_head = i % head_dim;
		float freq = j_head >= rotary_dim ? 0.f : 1.0f / powf(theta, (float)j_head / (float)rotary_dim);
		float val = pos * freq;
		float fcr = cosf(val);
		float fci = sinf(val);

		float v0 = vec[i];
		float v1 = vec[i + 1];
		vec[i] = v0 * fcr - v1 * fci;
		vec[i + 1] = v0 * fci + v1 * fcr;
	}
}

/* infer.cpp:216-248 */
void orc_attn(float *xout, float *atth, const float *qh, const uint16_t *kh, const uint16_t *vh, int head_dim,
              int n_kv_heads, int kv_len) {
	int kv_stride = n_kv_heads * head_dim;
	for (int t = 0; t < kv_len; ++t) {
		float score = 0.0f;
		for (int i = 0; i < head_dim; ++i) {
			score += qh[i] * half_to_float(kh[t * kv_stride + i]);
		}
		score /= sqrtf(head_dim);
		atth[t] = score;
	}
	softmax(atth, atth, kv_len);
	for (int i = 0; i < head_dim; ++i) {
		float vi = 0.0f;
		for (int t = 0; t < kv_len; ++t) {
			vi += atth[t] * half_to_float(vh[t * kv_stride + i]);
		}
		xout[i] = vi;
	}
}

/* infer.cpp:387-403 */
void orc_mha(float *xout, float *att, const uint16_t *kb, const uint16_t *vb, const float *q, int head_dim, int kv_len,
             int max_seq_len, int n_heads, int n_kv_heads) {
	int q_per_kv_head = n_heads / n_kv_heads;
	int h;
#pragma omp parallel for private(h)
	for (h = 0; h < n_heads; h++) {
		int kv_head_offset = (h / q_per_kv_head) * head_dim;
		orc_attn(xout + head_dim * h, att + max_seq_len * h, q + head_dim * h, kb + kv_head_offset,
		         vb + kv_head_offset, head_dim, n_kv_heads, kv_len);
	}
}

static void glu(float *hb, const float *hb2, int hidden_dim, int act) {
	if (act == 0) {
		for (int i = 0; i < hidden_dim; ++i) {
			hb[i] = gelu(hb[i]) * hb2[i];
		}
	} else {
		for (int i = 0; i < hidden_dim; ++i) {
			hb[i] = silu(hb[i]) * hb2[i];
		}
	}
}

/* infer.cpp:412-438 */
void orc_ffn(float *xout, const float *x, const void *w1, const void *w2, const void *w3, int hidden_dim, int dim,
             int act, int weight_dtype) {
	float *hb = (float *)malloc(sizeof(float) * hidden_dim);
	float *hb2 = (float *)malloc(sizeof(float) * hidden_dim);
	matmul_any(hb, x, w1, dim, hidden_dim, weight_dtype);
	matmul_any(hb2, x, w3, dim, hidden_dim, weight_dtype);
	glu(hb, hb2, hidden_dim, act);
	matmul_any(xout, hb, w2, hidden_dim, dim, weight_dtype);
	free(hb);
	free(hb2);
}

/* infer.cpp:254-385 (dense path: n_experts == 0, expert slot 0 with weight 1) */
void orc_block_forward(const orc_config *c, const orc_block *b, orc_state *s, int pos, int kv_sink, int kv_pos,
                       int kv_len) {
	int dt = c->weight_dtype;
	orc_rmsnorm(s->xb, s->x, b->rms_att, c->dim, c->norm_eps);

	int q_dim = c->n_heads * c->head_dim;
	int kv_dim = c->n_kv_heads * c->head_dim;

	matmul_any(s->q, s->xb, b->wq, c->dim, q_dim, dt);
	matmul_any(s->k, s->xb, b->wk, c->dim, kv_dim, dt);
	matmul_any(s->v, s->xb, b->wv, c->dim, kv_dim, dt);

	for (int i = 0; i < q_dim; ++i) {
		s->q[i] = clip(s->q[i], c->qkv_clip);
	}
	for (int i = 0; i < kv_dim; ++i) {
		s->k[i] = clip(s->k[i], c->qkv_clip);
		s->v[i] = clip(s->v[i], c->qkv_clip);
	}

	orc_rope(s->q, q_dim, c->head_dim, pos, c->rope_theta, c->rotary_dim);
	orc_rope(s->k, kv_dim, c->head_dim, pos, c->rope_theta, c->rotary_dim);

	uint16_t *kb = b->key_cache;
	uint16_t *vb = b->value_cache;
	for (int i = 0; i < kv_dim; ++i) {
		kb[(size_t)kv_pos * kv_dim + i] = float_to_half(s->k[i]);
		vb[(size_t)kv_pos * kv_dim + i] = float_to_half(s->v[i]);
	}

	/* infer.cpp:303-317: rotate attention-sink keys forward by one position */
	for (int r = 0; r < kv_sink; r++) {
		for (int i = 0; i < kv_dim; ++i) {
			s->k[i] = half_to_float(kb[r * kv_dim + i]);
		}
		orc_rope(s->k, kv_dim, c->head_dim, 1, c->rope_theta, c->rotary_dim);
		for (int i = 0; i < kv_dim; i++) {
			kb[r * kv_dim + i] = float_to_half(s->k[i]);
		}
	}

	int q_per_kv_head = c->n_heads / c->n_kv_heads;
	int h;
#pragma omp parallel for private(h)
	for (h = 0; h < c->n_heads; h++) {
		int kv_head_offset = (h / q_per_kv_head) * c->head_dim;
		orc_attn(s->xb2 + c->head_dim * h, s->att + (size_t)c->max_seq_len * h, s->q + c->head_dim * h,
		         kb + kv_head_offset, vb + kv_head_offset, c->head_dim, c->n_kv_heads, kv_len);
	}

	matmul_any(s->hb, s->xb2, b->wo, q_dim, c->dim, dt);
	for (int i = 0; i < c->dim; ++i) {
		s->x[i] += s->hb[i];
	}

	orc_rmsnorm(s->xb, s->x, b->rms_ffn, c->dim, c->norm_eps);

	matmul_any(s->hb, s->xb, b->w1, c->dim, c->hidden_dim, dt);
	matmul_any(s->hb2, s->xb, b->w3, c->dim, c->hidden_dim, dt);
	glu(s->hb, s->hb2, c->hidden_dim, c->act);
	matmul_any(s->xb2, s->hb, b->w2, c->hidden_dim, c->dim, dt);

	/* infer.cpp:377-383 with expert_weight = 1.0f (exact) */
	for (int i = 0; i < c->dim; ++i) {
		s->x[i] += s->xb2[i] * 1.0f;
	}
}

/* infer.cpp:483-485 */
void orc_kv_indices(int max_seq_len, int pos, int *kv_sink, int *kv_pos, int *kv_len) {
	int sink = pos >= max_seq_len ? 2 /* KV_SINKS, model.h:12 */ : 0;
	*kv_sink = sink;
	*kv_pos = sink + (pos - sink) % (max_seq_len - sink);
	*kv_len = pos >= max_seq_len ? max_seq_len : pos + 1;
}

/* infer.cpp:443-472, 474-523 */
void orc_forward(const orc_model *m, orc_state *s, int token, int pos, int mode) {
	const orc_config *c = &m->c;
	size_t off = (size_t)token * c->dim;
	switch (c->weight_dtype) {
	case 0:
		for (int i = 0; i < c->dim; ++i)
			s->x[i] = ((const float *)m->emb)[off + i];
		break;
	case 1:
		for (int i = 0; i < c->dim; ++i)
			s->x[i] = half_to_float(((const uint16_t *)m->emb)[off + i]);
		break;
	case 3:
		for (int i = 0; i < c->dim; ++i)
			s->x[i] = half_to_float((uint16_t)(((const uint8_t *)m->emb)[off + i] << 8));
		break;
	default:
		abort();
	}

	int kv_sink, kv_pos, kv_len;
	orc_kv_indices(c->max_seq_len, pos, &kv_sink, &kv_pos, &kv_len);
	for (int l = 0; l < c->n_layers; ++l) {
		orc_block_forward(c, &m->blocks[l], s, pos, kv_sink, kv_pos, kv_len);
	}
	if (mode == 0 /* HYDRATE_KV_CACHE */) {
		return;
	}
	orc_rmsnorm(s->x, s->x, m->rms_final, c->dim, c->norm_eps);
	matmul_any(s->logits, s->x, m->wcls, c->dim, c->vocab_size, c->weight_dtype);
	(void)dtype_size;
}

/* sampler.cpp:27-38: strict '>' so the first maximum wins */
int orc_sample_argmax(const float *logits, int vocab_size) {
	int argmax = 0;
	float max_val = -FLT_MAX;
	for (int i = 0; i < vocab_size; ++i) {
		if (logits[i] > max_val) {
			max_val = logits[i];
			argmax = i;
		}
	}
	return argmax;
}

/* sampler.cpp:11-25 */
float orc_sample_prob(const float *logits, int vocab_size, int index) {
	float max_val = -FLT_MAX;
	for (int i = 0; i < vocab_size; ++i) {
		if (logits[i] > max_val) {
			max_val = logits[i];
		}
	}
	float sum = 0;
	for (int i = 0; i < vocab_size; ++i) {
		sum += expf(logits[i] - max_val);
	}
	return expf(logits[index] - max_val) / sum;
}

/* sampler.cpp:6-9: the Sampler constructor seeds the C library generator */
void orc_srand(unsigned seed) {
	srand(seed);
}

/* sampler.cpp:40-65: temperature sampling by inverse CDF over softmax(logits / T) */
int orc_sample(const float *logits, int vocab_size, float temperature) {
	if (temperature == 0.0) {
		return orc_sample_argmax(logits, vocab_size);
	}
	float max_val = -FLT_MAX;
	for (int i = 0; i < vocab_size; ++i) {
		if (logits[i] > max_val) {
			max_val = logits[i];
		}
	}
	float sum = 0;
	for (int i = 0; i < vocab_size; ++i) {
		sum += expf((logits[i] - max_val) / temperature);
	}
	float r = rand() / (float)RAND_MAX;
	float cumsum = 0;
	for (int i = 0; i < vocab_size; ++i) {
		cumsum += expf((logits[i] - max_val) / temperature) / sum;
		if (cumsum >= r) {
			return i;
		}
	}
	return vocab_size - 1;
}

/* ---- synthetic weights: identical integer hash to yalm_amd/csrc/synth.hip ---- */
static inline uint64_t splitmix64(uint64_t x) {
	x += 0x9E3779B97F4A7C15ull;
	x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
	x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
	return x ^ (x >> 31);
}
/* uniform in [-scale, scale): 24 hash bits, integer-centred, one rounding */
static inline float synth_unit(uint64_t seed, uint64_t i, float k) {
	uint64_t h = splitmix64(seed ^ (i * 0xD1B54A32D192ED03ull));
	int32_t s = (int32_t)(h >> 40) - 8388608;
	return (float)s * k;
}

void orc_synth_f32(float *dst, size_t n, uint64_t seed, float scale, float offset) {
	const float k = scale * (1.0f / 8388608.0f);
	long long i;
#pragma omp parallel for schedule(static)
	for (i = 0; i < (long long)n; i++) {
		uint64_t h = splitmix64(seed ^ ((uint64_t)i * 0xD1B54A32D192ED03ull));
		int32_t s = (int32_t)(h >> 40) - 8388608;
		dst[i] = fmaf((float)s, k, offset);
	}
}

void orc_synth_f16(uint16_t *dst, size_t n, uint64_t seed, float scale) {
	const float k = scale * (1.0f / 8388608.0f);
	long long i;
#pragma omp parallel for schedule(static)
	for (i = 0; i < (long long)n; i++) {
		dst[i] = float_to_half(synth_unit(seed, (uint64_t)i, k));
	}
}

void orc_synth_f8(uint8_t *dst, size_t n, uint64_t seed, float scale) {
	const float k = scale * (1.0f / 8388608.0f);
	long long i;
#pragma omp parallel for schedule(static)
	for (i = 0; i < (long long)n; i++) {
		uint32_t h = float_to_half(synth_unit(seed, (uint64_t)i, k));
		/* round-to-nearest-even of the f16 bits to the top byte (E5M2) */
		dst[i] = (uint8_t)((h + 0x7Fu + ((h >> 8) & 1u)) >> 8);
	}
}

void orc_set_threads(int n) {
	omp_set_num_threads(n);
}
int orc_get_threads(void) {
	return omp_get_max_threads();
}
