// decoder.h — host-side state shared by the engine's translation units
// (yalm_hip.hip: shim, decoder, decode test API; prefill.hip: batched prefill).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/yalm_hip.h"
#include "device_common.h"
#include "tp_exchange.h"

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

// GEMV launch geometry of gemv_rb_kernel: threads, loads in flight per lane, workgroups per CU. 0 = automatic.
struct GemvCfg {
	int threads = 0, U = 0, gpw = 0;
};
enum { GK_QKV = 0, GK_WO = 1, GK_GLU = 2, GK_W2 = 3, GK_CLS = 4, GK_N = 5 };

int device_cu_count();

// Tuning / tracing knobs are read from the environment only in the A/B build
// (tools/build_ab_lib.sh compiles with -DYALM_AB): the production library's
// behaviour depends on none of them. Functional switches (separate attention and Wo
// launches; eager launches; a sync after every replay) are set per decoder through
// yalm_decoder_set_launch.
inline const char *ab_env(const char *name) {
#ifdef YALM_AB
	return getenv(name);
#else
	(void)name;
	return nullptr;
#endif
}

// Batched-prefill scratch (prefill.hip), allocated on first use for
// max_seq_len rows.
struct PrefillBufs {
	int cap = 0;
	float *X = nullptr;        // [cap][dim] f32 residual stream
	uint16_t *Xn = nullptr;    // [cap][2 dim] f16 normalised A operand ([hi | lo] before the QKV GEMM)
	uint16_t *Q = nullptr;     // [cap][q_dim] f16
	uint16_t *O = nullptr;     // [cap][q_dim] f16 attention output
	uint16_t *H = nullptr;     // [cap][hidden] f16 GLU output
	int *tok = nullptr;        // [cap] token ids
	int *tgt = nullptr;        // [cap] next-token targets (-1: none)
	float *pmax = nullptr, *psum = nullptr; // [cap][vocab / 128] logits partials
	float *tgt_logit = nullptr, *lp = nullptr; // [cap]
	float *rope = nullptr;                     // [cap][head_dim / 2][2]
	float *skp = nullptr;                      // split-K partials of the short-prompt GEMMs (prefill_skinny.h)
	size_t skp_floats = 0;
	unsigned *range = nullptr;                 // [n_layers + 1][4] f16-operand range guard (prefill.h range_note)
	uint16_t *wdq = nullptr;                   // fp8 models: one layer's (or the classifier's) weights as f16
	int last_passes = 0, last_scaled = 0;      // the last yalm_prefill: passes run, layers with a scaled GLU output
};

// Prefill GEMM forms (prefill.hip): per GEMM kind the large-tile width (-1 = auto,
// 128 / 192 / 256 / 320), the 8-phase schedule, the persistent tile loop. The defaults at
// decoder creation; other exact forms only through yalm_set_prefill_forms (the tests);
// never read from the environment by the production library.
struct PfForms {
	int g16[6] = {-1, -1, -1, -1, -1, -1}; // qkv, wo, glu, w2, cls, test
	bool p8 = true, persist = true;
	bool no_skinny = false; // T <= 64: split-K skinny GEMMs (prefill_skinny.h) unless set
	bool qkv1 = true;       // the q and k | v GEMMs as ONE two-depth launch when BN 256 fits both
	bool skl = true;        // skinny GEMMs: weight rows staged by LDS-DMA (prefill_skinny.h)
	bool split = false;     // split-operand precision form (yalm_set_prefill_precision): every f16
							// activation operand as [hi | lo], the large-tile GEMMs at every T
	bool wnorm = true;      // row norms: one wave per row, the row in registers (rmsnorm_rows_wave_kernel)
};
PfForms pf_forms_default(); // prefill.hip: the production forms (A/B build: YALM_PF_FORMS)

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
	float *x = nullptr, *q = nullptr, *xb2 = nullptr, *hb = nullptr, *logits = nullptr, *inv_freq = nullptr;
	unsigned long long *part = nullptr; // attention chunk partials as {value, tag} granules (attention.h)
	int *tokens = nullptr;
	int tokens_cap = 0;
	float *logits_pinned = nullptr;
	std::vector<void *> dev_allocs;
	hipGraph_t graph[N_GRAPHS] = {};
	hipGraphExec_t exec[N_GRAPHS] = {};
	long long host_pos = -1;         // position of the next forward as the host knows it (-1: unknown)
	GemvCfg gemv[GK_N];
	bool eager = false;     // YALM_LAUNCH_EAGER: launch kernels directly (profilers that mis-handle graph replay)
	// the device greedy loop (yalm_enqueue_greedy / yalm_generate_greedy) launches its forwards
	// directly rather than replaying GRAPH_GREEDY: measured 0.6-1.1% faster on MI355X in six
	// interleaved rounds (profiles/r5y_graph_vs_eager.txt); the host issues the 131 launches of
	// a token well inside the token's 1.6-2.5 ms. A/B builds: YALM_GREEDY_GRAPH=1 replays.
	bool greedy_eager = true;
	bool graph_sync = false; // YALM_LAUNCH_SYNC: synchronise after every replay
	std::string kname;
	PrefillBufs pf;
	PfForms pf_forms;
	// tensor parallelism (yalm_decoder_create_tp): c holds the LOCAL shard dims
	// (n_heads, n_kv_heads, hidden_dim, vocab_size divided by tp_size)
	int tp_rank = 0, tp_size = 1;
	void *comm = nullptr;            // ncclComm_t (RCCL); null = single-GPU decoder
	int vocab_full = 0;              // unsharded vocabulary (logits all-gather, host copies)
	float *xs = nullptr;             // [dim] Wo / W2 partial (+ x on rank 0), all-reduced into x
	float *logits_local = nullptr;   // [vocab / tp] this rank's logits rows (== logits without TP)
	float *amax = nullptr;           // [2] local argmax (value, global index as float bits)
	float *amax_all = nullptr;       // [2 * tp_size]
	// IPC transport (yalm_decoder_create_tp_ipc, tp_exchange.h): every rank's uncached
	// buffer [2 parities][tp_size][ipc_S floats][control words] mapped on all ranks; the
	// exchanges are folded into their producer and consumer kernels (no exchange launch)
	bool ipc = false;
	int ipc_S = 0;                   // floats per (parity, source) slot
	float *ipc_own = nullptr;        // this rank's buffer
	float **ipc_bufs = nullptr;      // device array [tp_size] of buffer bases (peers opened via IPC)
	std::vector<void *> ipc_opened;  // hipIpcOpenMemHandle mappings to close
	TpX tpx{};                       // the exchange descriptor passed to producers / consumers
	bool tpx_gate = false;           // ranks share this GPU: a 1-wave wait launch before each consumer
	bool tpx_collect = false;        // collect form (many ranks): a collect launch sums x before the consumer
	// launch path: attention + Wo as one launch (attn_wo.h) when supported (attn_wo_ok);
	// YALM_LAUNCH_SEPARATE_ATTN_WO selects the two separate kernels
	bool attn_wo = false, attn_wo_ok = false;
	int awo_nb = 0;                  // grid: n_kv * (awo_S + G - 1) attention + n_heads mergers + ceil(dim / AWO_RPW) Wo
	int awo_S = 0;                   // key-chunk splits per kv head
	int awo_slots = 0;               // co-resident workgroup slots of the fused launch (occupancy x CUs)
	unsigned long long *awo_trace = nullptr; // A/B build, YALM_ATTN_WO_TRACE=1: [grid][16] stamps of the last launch
	int awo_delay = 0;               // ticks the Wo workgroups wait before their slice loads
	// fp8 at kv_len <= AWO_SHORT_KV: no wait (round 5 sweep, profiles/r5aa_awo_delay_short.txt:
	// kv 17 / 32 / 64 7.72 / 7.43 / 7.56 us against 8.18 / 8.07 / 8.12 at 0.5 us, while kv 151 /
	// 401 keep the 0.5 us). The eager greedy loop knows each forward's kv_len from the host-side
	// position (awo_kv_hint); graph captures and unknown positions use awo_delay. A wrong hint
	// changes only the timing.
	int awo_delay_short = -1;        // -1: same as awo_delay
	long long awo_kv_hint = -1;      // kv_len of the forward being enqueued, -1 unknown
	unsigned long long *awo_gran = nullptr; // [n_layers][q_dim] attention outputs as {value, epoch} granules
	unsigned *awo_err = nullptr;     // error word of the in-launch waits (bit 0 fused Wo gather, bit 1 attention merger)
};

// ------------------------------------------------------------------ shared helpers
int dalloc(yalm_decoder_s *d, void **p, size_t bytes); // zeroed device allocation owned by d
int awo_check(yalm_decoder_s *d);                      // after a sync: a fused-launch spin that gave up
