// decoder.h — host-side state shared by the engine's translation units
// (yalm_hip.hip: shim, decoder, decode test API; prefill.hip: batched prefill).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/yalm_hip.h"
#include "device_common.h"
#include "engine.h"

// ------------------------------------------------------------------ errors
void set_err(const std::string &s); // yalm_hip.hip (thread-local last error)

#define HIPCHK(expr)                                                                                                   \
	do {                                                                                                               \
		hipError_t e_ = (expr);                                                                                        \
		if (e_ != hipSuccess) {                                                                                        \
			set_err(std::string(#expr) + " failed: " + hipGetErrorString(e_) + " (" + __FILE__ + ":" +                 \
			        std::to_string(__LINE__) + ")");                                                                   \
			return YALM_ERR_HIP;                                                                                       \
		}                                                                                                              \
	} while (0)

#define ARGCHK(cond, msg)                                                                                              \
	do {                                                                                                               \
		if (!(cond)) {                                                                                                 \
			set_err(msg);                                                                                              \
			return YALM_ERR_ARG;                                                                                       \
		}                                                                                                              \
	} while (0)

#define TRY(expr)                                                                                                      \
	do {                                                                                                               \
		int r_ = (expr);                                                                                               \
		if (r_ != YALM_OK)                                                                                             \
			return r_;                                                                                                 \
	} while (0)

// GEMV launch geometry (see gemv_stream_kernel). 0 = automatic.
struct GemvCfg {
	int threads = 0, U = 0, gpw = 0;
};
enum { GK_QKV = 0, GK_WO = 1, GK_GLU = 2, GK_W2 = 3, GK_CLS = 4, GK_N = 5 };

int device_cu_count();

// Work-stealing row-block GEMV (gemv_dyn.h, dyn.hip): launches policy P's GEMV
// with a static prefix + dequeued tail; DYN_FALLBACK when the shape does not fit
// (the caller then launches gemv_rb_kernel). ctr: DYN_SHARDS counters, zero at rest.
#define DYN_FALLBACK (-100)
template <class WT, class P, bool NORM>
int launch_dyn(const P &p, const float *x, const float *normw, float eps, unsigned *ctr, int frac_pct, hipStream_t st);

// Batched-prefill scratch (prefill.hip), allocated on first use for
// max_seq_len rows.
struct PrefillBufs {
	int cap = 0;
	float *X = nullptr;        // [cap][dim] f32 residual stream
	uint16_t *Xn = nullptr;    // [cap][dim] f16 normalised A operand
	uint16_t *Q = nullptr;     // [cap][q_dim] f16
	uint16_t *O = nullptr;     // [cap][q_dim] f16 attention output
	uint16_t *H = nullptr;     // [cap][hidden] f16 GLU output
	int *tok = nullptr;        // [cap] token ids
	int *tgt = nullptr;        // [cap] next-token targets (-1: none)
	float *pmax = nullptr, *psum = nullptr; // [cap][vocab / 128] logits partials
	float *tgt_logit = nullptr, *lp = nullptr; // [cap]
	float *rope = nullptr;                     // [cap][head_dim / 2][2]
};

// ------------------------------------------------------------------ decoder
enum { GRAPH_HYDRATE = 0, GRAPH_LOGITS = 1, GRAPH_GREEDY = 2, N_GRAPHS = 3 };

struct yalm_decoder_s {
	yalm_config c{};
	std::vector<yalm_block_weights> b;
	const void *emb = nullptr;
	const float *rms_final = nullptr;
	const void *wcls = nullptr;
	hipStream_t stream = nullptr;
	bool own_stream = false;
	StepState *step = nullptr;
	float *x = nullptr, *q = nullptr, *xb2 = nullptr, *hb = nullptr, *part = nullptr, *logits = nullptr,
	      *inv_freq = nullptr;
	int *tokens = nullptr;
	int tokens_cap = 0;
	float *logits_pinned = nullptr;
	std::vector<void *> dev_allocs;
	// [v][which]: v = 1 captures the short-context attention + Wo kernel (attn_wo_local_kernel)
	hipGraph_t graph[2][N_GRAPHS] = {};
	hipGraphExec_t exec[2][N_GRAPHS] = {};
	long long host_pos = -1;         // position of the next forward as the host knows it (-1: unknown)
	unsigned *attn_counters = nullptr; // per-kv-head arrival tickets (zeroed; the last arriver resets)
	GemvCfg gemv[GK_N];
	bool eager = false;     // YALM_EAGER=1: launch kernels directly (profilers that mis-handle graph replay)
	bool graph_sync = false; // YALM_GRAPH_SYNC=1: synchronise after every replay
	std::vector<void *> glu_il;      // YALM_GLU_INTERLEAVE=1: per layer [hidden][W1 row | W3 row] copies (device)
	int glu_w3_rot = 0;      // YALM_GLU_W3_ROT=1: W1|W3 GEMV streams W3 rows rotated by half (gemv.h rb_perm)
	int ablate = 0;          // YALM_ABLATE bitmask: skip qkv|attn|wo|glu|w2 (1|2|4|8|16), or (32) load no Wo
	                         // weights in the fused attention + Wo launch; timing only, results wrong
	std::string kname;
	PrefillBufs pf;
	// tensor parallelism (yalm_decoder_create_tp): c holds the LOCAL shard dims
	// (n_heads, n_kv_heads, hidden_dim, vocab_size divided by tp_size)
	int tp_rank = 0, tp_size = 1;
	void *comm = nullptr;            // ncclComm_t (RCCL); null = single-GPU decoder
	int vocab_full = 0;              // unsharded vocabulary (logits all-gather, host copies)
	float *xs = nullptr;             // [dim] Wo / W2 partial (+ x on rank 0), all-reduced into x
	float *logits_local = nullptr;   // [vocab / tp] this rank's logits rows (== logits without TP)
	float *amax = nullptr;           // [2] local argmax (value, global index as float bits)
	float *amax_all = nullptr;       // [2 * tp_size]
	// IPC one-shot exchange transport (yalm_decoder_create_tp_ipc): every rank's
	// buffer [2 slots x ipc_S floats][flags: 64 u32][seq u32] mapped on all ranks
	bool ipc = false;
	int ipc_S = 0;                   // floats per slot
	float *ipc_own = nullptr;        // this rank's buffer
	float **ipc_bufs = nullptr;      // device array [tp_size] of buffer bases (peers opened via IPC)
	std::vector<void *> ipc_opened;  // hipIpcOpenMemHandle mappings to close
	// persistent per-token engine (engine.h): one launch per token when the
	// config is supported (single GPU, head_dim 128, G <= 4, dims multiple of
	// 64 * EPL and <= 16384); YALM_ENGINE=0 selects the launch path
	bool engine = false;
	int eng_nb = 0;                  // workgroups = CUs
	EngLayer *eng_layers = nullptr;  // [n_layers]
	unsigned *eng_flags = nullptr;   // [round_up(NB, 256)] per-CU epochs
	unsigned *eng_gen = nullptr;     // launch generation
	unsigned *eng_err = nullptr;     // error bits (ENG_ERR_*)
	unsigned *eng_tickets = nullptr; // [n_kv] attention arrival tickets
	float *eng_part = nullptr;       // [n_heads][ENG_SMAX][head_dim + 2] split partials
	float *eng_amax = nullptr;       // [NB][2] per-CU (max, index)
	EngArgs *eng_args = nullptr;     // [N_GRAPHS] kernel arguments per mode (device)
	unsigned long long *eng_trace = nullptr; // YALM_ENGINE_TRACE=1: [NB][5 L + 2][8] stamps
	// launch path: attention + Wo as one launch (attn_wo.h) when supported;
	// YALM_ATTN_WO=0 selects the two separate kernels
	bool attn_wo = false;
	int awo_nb = 0;                  // grid: n_kv * awo_S attention + ceil(dim / AWO_RPW) Wo workgroups
	int awo_S = 0;                   // key-chunk splits per kv head
	unsigned long long *awo_trace = nullptr; // YALM_ATTN_WO_TRACE=1: [grid][4] stamps of the last launch
	int awo_win = 0;                 // Wo loads in flight per lane (YALM_ATTN_WO_WIN), -1 = none (ablation)
	int awo_delay = 0;
	int awo_spec = 0;                // YALM_AWO_SPEC=1: speculative gather after the slice landed (attn_wo.h)               // ticks the Wo workgroups wait before their slice loads (YALM_ATTN_WO_DELAY)
	unsigned long long *awo_gran = nullptr; // [n_layers][q_dim] attention outputs as {value, epoch} granules
	unsigned *awo_err = nullptr;     // error word (bounded spins that gave up)
	int awo_local_max = 0;           // kv_len up to which the short-context kernel runs (YALM_AWO_LOCAL, 0 = never)
	bool awo_local_now = false;      // the forward being enqueued uses attn_wo_local_kernel
	int awl_kv_first = 1;            // YALM_AWL_KV_FIRST: K/V loads issued ahead of the Wo slice
	unsigned long long *awl_trace = nullptr; // YALM_ATTN_WO_TRACE=1: [dim / 16][4] stamps of the last local launch
	// launch path: rmsnorm + GLU + W2 + residual as one launch (ffn.h) when
	// supported; YALM_FFN=0 selects the separate GLU and W2 kernels
	bool ffn = false;
	int ffn_nb = 0;                  // workgroups = CUs (all co-resident)
	int ffn_P = 8;                   // extra W2 loads in flight per wave across the seam (YALM_FFN_P)
	size_t ffn_lds = 0;              // dynamic LDS bytes
	unsigned *ffn_flags = nullptr;   // [n_layers][ffn_nb] per-workgroup epochs, then the error word
	unsigned *ffn_err = nullptr;
	unsigned long long *ffn_trace = nullptr; // YALM_FFN_TRACE=1: [ffn_nb][8] stamps of the last launch
	// work-stealing tail for the weight-streaming GEMVs (gemv_dyn.h), opt-in YALM_DYN=1
	// (slower than the static row-block kernel as measured); YALM_DYN_FRAC = percent pooled
	bool dyn = false;
	int dyn_frac = 10;
	unsigned *dyn_ctr = nullptr;     // DYN_SHARDS counters, 32 words apart (self-resetting per launch)
};

// ------------------------------------------------------------------ shared helpers
int dalloc(yalm_decoder_s *d, void **p, size_t bytes); // zeroed device allocation owned by d

// short-context fused attention + Wo (awl.hip, attn_wo_local.h)
int attn_wo_local_occupancy(int dtype, int G, int XS); // workgroups per CU (0: not launchable)
int launch_attn_wo_local(yalm_decoder_s *d, const yalm_block_weights &w);

// persistent engine (engine.hip)
int engine_init(yalm_decoder_s *d);                // enables d->engine when supported
int engine_enqueue(yalm_decoder_s *d, int which);  // one launch = one token (graph `which`)
int engine_check(yalm_decoder_s *d);               // after a sync: bounded spins that gave up
