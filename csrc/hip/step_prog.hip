// Native step runner: the HIP executor's training step as a flat op list
// (kernel launches on 4 streams, event record / wait edges), issued from C++
// for a whole block of steps per host call.
//
// The step (gentun_amd/models/cnn_hip.py HipPopJob._step_plan) is fixed once a
// job's argument tables exist: every launch reads its per-step state (global
// step, shuffle position, learning rate) from device memory, so the same op
// list is valid for every step. The Python issue path costs ~20 us per launch
// and the captured HIP graph replays the multi-stream step 2-12 % slower than
// the same launches issued eagerly (profiles/graph_vs_eager_ab_r4.txt); this
// runner issues them at C++ cost.
//
// Reference parity: the reference trains each fold with Keras model.fit
// (/root/reference/gentun/models/keras_models.py:127-143); this is the
// executor of that loop for a whole population of folds.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

extern "C" {
// launch entry points of the other translation units (same library)
int gt_step_begin(void* st, hipStream_t s);
int gt_conv_fwd(const void* a, hipStream_t s);
int gt_conv_wgrad(const void* a, hipStream_t s);
int gt_wgrad_reduce(const void* a, hipStream_t s);
int gt_bn_fwd(const void* a, hipStream_t s);
int gt_bn_bwd(const void* a, hipStream_t s);
int gt_dense_fwd(const void* a, hipStream_t s);
int gt_head(const void* a, hipStream_t s);
int gt_dense_dgrad(const void* a, hipStream_t s);
int gt_dense_wgrad_adam(const void* a, hipStream_t s);
int gt_adam_segments(const void* a, int nblocks, hipStream_t s);
int gt_pool_fwd(const void* x0, const void* x1, const int* sel, void* y, int NB, int B, int H, int W, int Cp,
                int prec, hipStream_t s);
int gt_pool_fwd_mask(const void* x0, const void* x1, const int* sel, void* y, int NB, int B, int H, int W, int Cp,
                     uint8_t* mask, int prec, hipStream_t s);
int gt_pool_bwd_mask(const uint8_t* mask, const int* sel, const void* dy, void* dx0, void* dx1, int NB, int B,
                     int H, int W, int Cp, int relu_mask, int prec, hipStream_t s);
int gt_wino_wtrans(const void* a, int nblocks, hipStream_t s);
int gt_conv_wfrag(const void* a, int nblocks, hipStream_t s);
}

namespace {

// op kinds (gentun_amd/ops/cnn_kernels.py PROG_OPS mirrors this list)
enum : int32_t {
  OP_RECORD = 0, OP_WAIT = 1, OP_STEP_BEGIN = 2, OP_CONV = 3, OP_WGRAD = 4, OP_WGRAD_REDUCE = 5,
  OP_BN_FWD = 6, OP_BN_BWD = 7, OP_DENSE_FWD = 8, OP_HEAD = 9, OP_DENSE_DGRAD = 10, OP_DENSE_WGRAD_ADAM = 11,
  OP_ADAM = 12, OP_POOL_FWD = 13, OP_POOL_FWD_MASK = 14, OP_POOL_BWD_MASK = 15, OP_WINO_WTRANS = 16, OP_CONV_WFRAG = 17, OP_COUNT = 18
};

constexpr int kMaxV = 14;

}  // namespace

// one op: kind, stream index, event index (record / wait), then operands:
// v[0] = argument-struct address (struct launches) or the positional operands
// (pool launches: pointers and ints in signature order)
struct GtProgOp {
  int32_t kind, stream, event, pad;
  int64_t v[kMaxV];
};

struct GtProg {
  std::vector<GtProgOp> ops;
  std::vector<hipEvent_t> ev;
  int nstreams = 0;
};

static inline void* P(int64_t x) { return reinterpret_cast<void*>(static_cast<intptr_t>(x)); }
static inline int I(int64_t x) { return static_cast<int>(x); }

static int run_op(const GtProg& p, const GtProgOp& o, const hipStream_t* streams) {
  hipStream_t s = streams[o.stream];
  const int64_t* v = o.v;
  switch (o.kind) {
    case OP_RECORD: return (int)hipEventRecord(p.ev[o.event], s);
    case OP_WAIT: return (int)hipStreamWaitEvent(s, p.ev[o.event], 0);
    case OP_STEP_BEGIN: return gt_step_begin(P(v[0]), s);
    case OP_CONV: return gt_conv_fwd(P(v[0]), s);
    case OP_WGRAD: return gt_conv_wgrad(P(v[0]), s);
    case OP_WGRAD_REDUCE: return gt_wgrad_reduce(P(v[0]), s);
    case OP_BN_FWD: return gt_bn_fwd(P(v[0]), s);
    case OP_BN_BWD: return gt_bn_bwd(P(v[0]), s);
    case OP_DENSE_FWD: return gt_dense_fwd(P(v[0]), s);
    case OP_HEAD: return gt_head(P(v[0]), s);
    case OP_DENSE_DGRAD: return gt_dense_dgrad(P(v[0]), s);
    case OP_DENSE_WGRAD_ADAM: return gt_dense_wgrad_adam(P(v[0]), s);
    case OP_ADAM: return gt_adam_segments(P(v[0]), I(v[1]), s);
    case OP_WINO_WTRANS: return gt_wino_wtrans(P(v[0]), I(v[1]), s);
    case OP_CONV_WFRAG: return gt_conv_wfrag(P(v[0]), I(v[1]), s);
    case OP_POOL_FWD:
      return gt_pool_fwd(P(v[0]), P(v[1]), static_cast<const int*>(P(v[2])), P(v[3]), I(v[4]), I(v[5]), I(v[6]),
                         I(v[7]), I(v[8]), I(v[9]), s);
    case OP_POOL_FWD_MASK:
      return gt_pool_fwd_mask(P(v[0]), P(v[1]), static_cast<const int*>(P(v[2])), P(v[3]), I(v[4]), I(v[5]),
                              I(v[6]), I(v[7]), I(v[8]), static_cast<uint8_t*>(P(v[9])), I(v[10]), s);
    case OP_POOL_BWD_MASK:
      return gt_pool_bwd_mask(static_cast<const uint8_t*>(P(v[0])), static_cast<const int*>(P(v[1])), P(v[2]),
                              P(v[3]), P(v[4]), I(v[5]), I(v[6]), I(v[7]), I(v[8]), I(v[9]), I(v[10]), I(v[11]), s);
    default: return -100;
  }
}

extern "C" {

size_t gt_sizeof_prog_op() { return sizeof(GtProgOp); }

void gt_prog_destroy(void* h) {
  GtProg* p = static_cast<GtProg*>(h);
  if (!p) return;
  for (hipEvent_t e : p->ev)
    if (e) (void)hipEventDestroy(e);
  delete p;
}

// Validates every op (kind, stream and event indices in range, every event
// recorded before it is waited on) and creates the events. nullptr on error.
void* gt_prog_create(const GtProgOp* ops, int n, int nevents, int nstreams) {
  if (n <= 0 || nevents < 0 || nstreams <= 0) return nullptr;
  std::vector<char> recorded(nevents, 0);
  for (int i = 0; i < n; ++i) {
    const GtProgOp& o = ops[i];
    if (o.kind < 0 || o.kind >= OP_COUNT || o.stream < 0 || o.stream >= nstreams) return nullptr;
    if (o.kind == OP_RECORD || o.kind == OP_WAIT) {
      if (o.event < 0 || o.event >= nevents) return nullptr;
      if (o.kind == OP_RECORD) recorded[o.event] = 1;
      else if (!recorded[o.event]) return nullptr;
    } else if (o.v[0] == 0) {
      return nullptr;                                  // every launch has an argument block / first operand
    }
  }
  GtProg* p = new GtProg;
  p->ops.assign(ops, ops + n);
  p->nstreams = nstreams;
  p->ev.assign(nevents, nullptr);
  for (auto& e : p->ev) {
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      e = nullptr;
      gt_prog_destroy(p);
      return nullptr;
    }
  }
  return p;
}

// Issues the op list nsteps times on streams[0 .. nstreams-1] (streams[0]:
// the caller's stream). Returns 0, or the failing launch's code with its op
// index in *failed_op.
int gt_prog_run(void* h, const hipStream_t* streams, int nsteps, int* failed_op) {
  const GtProg* p = static_cast<const GtProg*>(h);
  if (!p || !streams) return -101;
  for (int step = 0; step < nsteps; ++step) {
    for (size_t i = 0; i < p->ops.size(); ++i) {
      const int rc = run_op(*p, p->ops[i], streams);
      if (rc != 0) {
        if (failed_op) *failed_op = (int)i;
        return rc;
      }
    }
  }
  return 0;
}

}  // extern "C"
