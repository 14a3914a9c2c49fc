// C ABI entry points (include/fia.h).  Validates arguments, keeps the context
// state machine (params -> index -> prepare -> query), converts HIP errors to
// status codes + a message, and never lets an exception cross the boundary.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>

#include "common.h"

namespace fia {

static bool pooled_event(fia_ctx* c, hipEvent_t* e) {
  if (!c->events.pool.empty()) {
    *e = c->events.pool.back();
    c->events.pool.pop_back();
    return true;
  }
  return hipEventCreate(e) == hipSuccess;
}

void phase_begin(fia_ctx* c, int phase, hipStream_t s) {
  if (!(c->profiling >> phase & 1u)) return;
  hipEvent_t a, b;
  if (!pooled_event(c, &a)) return;
  if (!pooled_event(c, &b)) { c->events.pool.push_back(a); return; }
  (void)hipEventRecord(a, s);
  c->events.ev[phase].push_back({a, b});
}

void phase_end(fia_ctx* c, int phase, hipStream_t s) {
  if (!(c->profiling >> phase & 1u) || c->events.ev[phase].empty()) return;
  (void)hipEventRecord(c->events.ev[phase].back().second, s);
}

PhaseSpan phase_span(fia_ctx* c, int phase) {
  PhaseSpan ps;
  if (!(c->profiling >> phase & 1u)) return ps;
  hipEvent_t a, b;
  if (!pooled_event(c, &a)) return ps;
  if (!pooled_event(c, &b)) { c->events.pool.push_back(a); return ps; }
  c->events.ev[phase].push_back({a, b});
  ps.a = a;
  ps.b = b;
  return ps;
}

// The stream a small-k Gram pass runs on: the context's aux stream, made to wait for
// everything queued on `s` so far; `s` itself while `s` is being captured into a graph (a
// fork there would have to be joined inside the same capture) or when aux is unavailable.
hipStream_t prepare_stream(fia_ctx* c, hipStream_t s) {
  // MF k <= 16: the query scans the fork would overlap (~20 us at ml-1m-ex) barely exceed the
  // cross-queue wait of the join (~10 us on MI355X), and they run slower beside the Gram pass:
  // same-box A/B 0.172-0.173 ms per ml-1m-ex step on one stream vs 0.176-0.182 forked
  if (c->p.model == FIA_MODEL_MF && c->p.k <= 16) return s;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return s;
  if (!c->aux) {
    // the stream and its three events all or nothing (a half-made set would fork work that
    // can never be joined)
    hipStream_t a = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool ok = hipStreamCreateWithFlags(&a, hipStreamNonBlocking) == hipSuccess;
    for (int t = 0; t < 3 && ok; ++t) ok = hipEventCreateWithFlags(&ev[t], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
      if (a) (void)hipStreamDestroy(a);
      return s;
    }
    c->aux = a;
    c->fork_ev = ev[0];
    c->prep_ev = ev[1];
    c->l1_ev = ev[2];
  }
  if (hipEventRecord(c->fork_ev, s) != hipSuccess || hipStreamWaitEvent(c->aux, c->fork_ev, 0) != hipSuccess) return s;
  return c->aux;
}

// after the pass was queued on ps: the point later consumers on the caller's stream join.
// Called after a failed pass too: the kernels already queued on ps are joined by the next call
// (or, when even the record fails, waited for here) before any buffer they read can be regrown.
hipError_t prepare_record(fia_ctx* c, hipStream_t ps, hipStream_t s) {
  if (ps == s) return hipSuccess;
  hipError_t e = hipEventRecord(c->prep_ev, ps);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(ps);
    return e;
  }
  c->prep_pending = true;
  return hipSuccess;
}

hipError_t join_prepare(fia_ctx* c, hipStream_t s) {
  c->l1_pending = false;           // recorded before prep_ev on the same stream
  if (!c->prep_pending) return hipSuccess;
  FIA_HIP_TRY(hipStreamWaitEvent(s, c->prep_ev, 0));
  c->prep_pending = false;
  return hipSuccess;
}

hipError_t join_l1(fia_ctx* c, hipStream_t s) {
  if (!c->l1_pending) return join_prepare(c, s);
  FIA_HIP_TRY(hipStreamWaitEvent(s, c->l1_ev, 0));
  c->l1_pending = false;
  return hipSuccess;
}

}  // namespace fia

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int fail(fia_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(fia_ctx* c, hipError_t e, const char* where) {
  return fail(c, FIA_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define FIA_GUARDED(ctx, ...)                                          \
  try {                                                                \
    __VA_ARGS__                                                        \
  } catch (const std::bad_alloc&) {                                    \
    return fail(ctx, FIA_ERR_NOMEM, "host allocation failed");         \
  } catch (...) {                                                      \
    return fail(ctx, FIA_ERR_INVALID, "unexpected internal exception"); \
  }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Every stream-taking entry point starts here.  DevBuf regrows free their old block in
// order on the CALLING stream; when the caller switches streams, kernels of the previous
// call may still be queued on the old one, so that stream is synchronised first (rare: a
// context normally sees one stream).  Only the context's own previous stream is waited for
// -- never the whole device, which would also wait for (and, in global capture mode,
// invalidate a capture on) other contexts' streams.  A previous stream that is capturing
// cannot be synchronised; nothing of ours can be freed under it (DevBuf::reserve refuses to
// regrow during a capture).
// A capture cannot start while a Gram pass forked onto the context's aux stream by an eager
// fia_prepare / fia_prepare_for is still unjoined: the captured kernels would have no edge to
// it (an event recorded outside the capture is no graph dependency, and no host wait is legal
// inside a global-mode capture), so a replay could read Gram caches still being written.
// That call fails with FIA_ERR_STATE; a joining call (fia_query_batch or fia_prepare) on a
// non-capturing stream clears the condition.
int enter_stream(fia_ctx* c, hipStream_t s, const char* where) {
  hipStreamCaptureStatus ns = hipStreamCaptureStatusNone;
  const bool new_capturing = hipStreamIsCapturing(s, &ns) == hipSuccess && ns != hipStreamCaptureStatusNone;
  if (new_capturing && c->prep_pending)
    return fail(c, FIA_ERR_STATE,
                std::string(where) + ": a forked Gram pass of an earlier eager fia_prepare is not joined yet; "
                "call fia_query_batch (or fia_prepare) on a non-capturing stream before starting a capture");
  if (c->has_stream && c->stream != s) {
    if (hipError_t e = fia::join_prepare(c, c->stream); e != hipSuccess) return hip_fail(c, e, where);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    // a capture starting on a new stream (a graph captured after eager warm-up on another
    // stream): no synchronisation is legal inside a global-mode capture, and none is needed
    // -- nothing can be regrown, so nothing freed, while capturing; the caller has finished
    // the warm-up stream (fia.h)
    if (!new_capturing && hipStreamIsCapturing(c->stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
      if (hipError_t e = hipStreamSynchronize(c->stream); e != hipSuccess) return hip_fail(c, e, where);
    }
  }
  c->stream = s;
  c->has_stream = true;
  return FIA_OK;
}

// contexts alive per device (fia_create / fia_destroy)
constexpr int kMaxDevices = 64;
std::atomic<int> g_live[kMaxDevices];

}  // namespace

namespace fia {
int live_contexts(int device) { return device >= 0 && device < kMaxDevices ? g_live[device].load() : 1; }
}  // namespace fia

extern "C" {

int fia_version(void) { return 100; }

int fia_create(int device, fia_ctx** out) {
  if (!out) return FIA_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return FIA_ERR_HIP;
  if (device < 0 || device >= n) return FIA_ERR_INVALID;
  fia_ctx* c = new (std::nothrow) fia_ctx();
  if (!c) return FIA_ERR_NOMEM;
  c->device = device;
  if (device < kMaxDevices) g_live[device].fetch_add(1);
  *out = c;
  return FIA_OK;
}

int fia_destroy(fia_ctx* c) {
  if (!c) return FIA_OK;
  {
    DeviceGuard g(c->device);
    // Only the context's own streams are waited for -- never the whole device, which would
    // also wait for (and, in global capture mode, invalidate a capture on) other streams.
    // The buffers are freed in order on the context's stream, then that stream is synchronised
    // so the frees complete before the context goes.  A context that never saw a stream owns
    // no device buffer.  (Destroying a context while its stream is being captured leaves its
    // buffers to the pool: they cannot be freed inside someone else's capture.)
    const hipStream_t ds = c->has_stream ? c->stream : nullptr;
    hipStreamCaptureStatus dcs = hipStreamCaptureStatusNone;
    const bool capturing = c->has_stream && !(hipStreamIsCapturing(ds, &dcs) == hipSuccess &&
                                              dcs == hipStreamCaptureStatusNone);
    const bool can_free = c->has_stream && !capturing;
    // (inside a capture no host wait is legal: the aux stream, like the buffers, is left)
    if (c->aux && !capturing) (void)hipStreamSynchronize(c->aux);
    c->prep_pending = c->l1_pending = false;
    if (can_free) (void)hipStreamSynchronize(ds);
    auto rel = [&](fia::DevBuf& b) {
      if (can_free) b.release(ds);
      else { b.ptr = nullptr; b.bytes = 0; }
    };
    for (int s = 0; s < 2; ++s) {
      for (fia::DevBuf* b : {&c->idx.side[s].ptr, &c->idx.side[s].row, &c->idx.side[s].other, &c->idx.side[s].rating,
                             &c->gram[s], &c->l1[s], &c->idx.order[s], &c->idx.gitems[s], &c->idx.gcomb[s],
                             &c->gpart[s], &c->self[s], &c->gm[s], &c->slot[s], &c->bitems[s], &c->bcomb[s]})
        rel(*b);
    }
    fia::DevBuf* bufs[] = {&c->rec,    &c->coff,   &c->cdesc,    &c->cand_pos,  &c->cand_val, &c->qscan,
                           &c->flag,   &c->nch,    &c->coupled,  &c->idx.pkey,  &c->idx.pcnt, &c->idx.psum,
                           &c->gcnt,   &c->gstart, &c->grank,    &c->gq,        &c->qbase,    &c->gscan,
                           &c->wstart, &c->witems, &c->resid,  &c->qwork,  &c->xb,       &c->syslist,
                           &c->cpllist, &c->lscr, &c->mark, &c->d1tab, &c->slices, &c->wfrag};
    for (auto* b : bufs) rel(*b);
    if (can_free) (void)hipStreamSynchronize(ds);   // the stream-ordered frees complete
    if (c->aux && !capturing) (void)hipStreamDestroy(c->aux);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->l1_ev) (void)hipEventDestroy(c->l1_ev);
    if (c->prep_ev) (void)hipEventDestroy(c->prep_ev);
    for (auto& v : c->events.ev)
      for (auto& pr : v) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto e : c->events.pool) (void)hipEventDestroy(e);
  }
  if (c->device >= 0 && c->device < kMaxDevices) g_live[c->device].fetch_sub(1);
  delete c;
  return FIA_OK;
}

const char* fia_last_error(const fia_ctx* c) { return c ? c->err.c_str() : ""; }

int fia_num_params(const fia_ctx* c) {
  if (!c || !c->p.valid) return 0;
  return fia::model_num_params(c->p.model, c->p.k);
}

int fia_set_params(fia_ctx* c, int model, int k, int64_t U, int64_t I, const float* const* tables, int nptrs,
                   double wd, double damping) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    // a small-k Gram pass still queued on the aux stream reads the tables being replaced
    // (this call has no stream to order behind it: wait for the pass on the host)
    if (c->prep_pending && c->aux) {
      DeviceGuard g(c->device);
      if (hipError_t es = hipStreamSynchronize(c->aux); es != hipSuccess) return hip_fail(c, es, "fia_set_params");
      c->prep_pending = c->l1_pending = false;
    }
    if (model != FIA_MODEL_MF && model != FIA_MODEL_NCF) return fail(c, FIA_ERR_INVALID, "unknown model");
    const int need = model == FIA_MODEL_MF ? 5 : 10;
    if (!tables || nptrs != need) return fail(c, FIA_ERR_INVALID, "wrong number of parameter tables");
    for (int t = 0; t < need; ++t)
      if (!tables[t]) return fail(c, FIA_ERR_INVALID, "null parameter table");
    if (U <= 0 || I <= 0 || U >= (1LL << 31) || I >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "bad table sizes");
    if (!fia::model_supported(model, k))
      return fail(c, FIA_ERR_UNSUPPORTED, "embedding size " + std::to_string(k) + " not built for this model");
    if (!(wd >= 0.0) || !(damping >= 0.0)) return fail(c, FIA_ERR_INVALID, "weight_decay/damping must be >= 0");
    if (c->idx.valid && (c->idx.U != U || c->idx.I != I))
      return fail(c, FIA_ERR_INVALID, "num_users/num_items differ from the built index");
    c->p.model = model;
    c->p.k = k;
    c->p.U = U;
    c->p.I = I;
    for (int t = 0; t < 10; ++t) c->p.t[t] = t < need ? tables[t] : nullptr;
    c->p.wd = wd;
    c->p.damping = damping;
    c->p.valid = true;
    c->prepared = false;
    return FIA_OK;
  })
}

int fia_build_index(fia_ctx* c, int64_t N, int64_t U, int64_t I, const int32_t* user, const int32_t* item,
                    const float* rating, void* stream) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    if (N < 0 || N >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "n_train out of range");
    if (U <= 0 || I <= 0 || U >= (1LL << 31) || I >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "bad entity counts");
    if (N > 0 && (!user || !item || !rating)) return fail(c, FIA_ERR_INVALID, "null training array");
    if (c->p.valid && (c->p.U != U || c->p.I != I))
      return fail(c, FIA_ERR_INVALID, "num_users/num_items differ from the registered params");
    DeviceGuard g(c->device);
    if (int rc = enter_stream(c, as_stream(stream), "fia_build_index"); rc != FIA_OK) return rc;
    if (hipError_t es = fia::join_prepare(c, as_stream(stream)); es != hipSuccess) return hip_fail(c, es, "fia_build_index");
    std::string why;
    hipError_t e = fia::build_index(c, N, U, I, user, item, rating, as_stream(stream), why);
    c->prepared = false;
    if (e != hipSuccess) {
      if (!why.empty()) return fail(c, FIA_ERR_INVALID, why);
      return hip_fail(c, e, "fia_build_index");
    }
    return FIA_OK;
  })
}

int fia_prepare(fia_ctx* c, void* stream) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    if (!c->p.valid) return fail(c, FIA_ERR_STATE, "fia_set_params has not been called");
    if (!c->idx.valid) return fail(c, FIA_ERR_STATE, "fia_build_index has not been called");
    DeviceGuard g(c->device);
    hipStream_t s = as_stream(stream);
    if (int rc = enter_stream(c, s, "fia_prepare"); rc != FIA_OK) return rc;
    if (hipError_t es = fia::join_prepare(c, s); es != hipSuccess) return hip_fail(c, es, "fia_prepare");
    bool unsup = false;
    // small k: the Gram pass on the aux stream (the large-k prepare synchronises inside)
    const hipStream_t ps = fia::big_supported(c->p.model, c->p.k) ? s : fia::prepare_stream(c, s);
    fia::phase_begin(c, 0, ps);
    hipError_t e = fia::prepare_model(c, ps, unsup);
    fia::phase_end(c, 0, ps);
    if (hipError_t er = fia::prepare_record(c, ps, s); e == hipSuccess) e = er;
    c->prepared = false;
    if (unsup) return fail(c, FIA_ERR_UNSUPPORTED, "model/k not supported");
    if (e == hipErrorOutOfMemory) return fail(c, FIA_ERR_NOMEM, "device memory exhausted by the Hessian caches");
    if (e != hipSuccess) return hip_fail(c, e, "fia_prepare");
    c->prepared = true;
    return FIA_OK;
  })
}

int fia_prepare_for(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, void* stream) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    if (!c->p.valid) return fail(c, FIA_ERR_STATE, "fia_set_params has not been called");
    if (!c->idx.valid) return fail(c, FIA_ERR_STATE, "fia_build_index has not been called");
    if (Q < 0 || Q >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "num_queries out of range");
    if (Q > 0 && (!qu || !qi)) return fail(c, FIA_ERR_INVALID, "null query array");
    DeviceGuard g(c->device);
    hipStream_t s = as_stream(stream);
    if (int rc = enter_stream(c, s, "fia_prepare_for"); rc != FIA_OK) return rc;
    // the marks below are read by a still-queued Gram pass
    if (hipError_t es = fia::join_prepare(c, s); es != hipSuccess) return hip_fail(c, es, "fia_prepare_for");
    bool unsup = false;
    hipError_t e;
    if (fia::big_supported(c->p.model, c->p.k)) {
      fia::phase_begin(c, 0, s);
      e = fia::prepare_big(c, Q, qu, qi, s);
      fia::phase_end(c, 0, s);
    } else {
      // small k: entities marked on s (no sync), their Gram caches on the aux stream
      fia::phase_begin(c, 0, s);
      e = fia::prepare_model_for(c, Q, qu, qi, s, s, unsup, true);
      const hipStream_t ps = e == hipSuccess ? fia::prepare_stream(c, s) : s;
      if (e == hipSuccess && !unsup) e = fia::prepare_model_for(c, Q, qu, qi, s, ps, unsup, false);
      fia::phase_end(c, 0, ps);
      if (hipError_t er = fia::prepare_record(c, ps, s); e == hipSuccess) e = er;
    }
    c->prepared = false;
    if (unsup) return fail(c, FIA_ERR_UNSUPPORTED, "model/k not supported");
    if (e == hipErrorOutOfMemory) return fail(c, FIA_ERR_NOMEM, "device memory exhausted by the Hessian caches");
    if (e != hipSuccess) return hip_fail(c, e, "fia_prepare_for");
    c->prepared = true;
    return FIA_OK;
  })
}

int fia_count_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int64_t* offsets,
                      int64_t* total_out, void* stream) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    if (!c->idx.valid) return fail(c, FIA_ERR_STATE, "fia_build_index has not been called");
    if (Q < 0 || Q >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "num_queries out of range");
    if (!offsets || (Q > 0 && (!qu || !qi))) return fail(c, FIA_ERR_INVALID, "null query array");
    DeviceGuard g(c->device);
    hipStream_t s = as_stream(stream);
    if (int rc = enter_stream(c, s, "fia_count_related"); rc != FIA_OK) return rc;
    hipError_t e = hipSuccess;
    if (total_out) {
      e = c->flag.reserve(64, s);
      if (e != hipSuccess) return hip_fail(c, e, "fia_count_related");
      e = hipMemsetAsync(c->flag.ptr, 0, 64, s);
      if (e != hipSuccess) return hip_fail(c, e, "fia_count_related");
    }
    e = fia::count_related(c, Q, qu, qi, offsets, s);
    if (e == hipSuccess && total_out) e = fia::check_cover(c, Q, qu, qi, c->flag.as<int32_t>() + 2, s);
    if (e == hipSuccess && total_out) e = fia::check_cover_small(c, Q, qu, qi, c->flag.as<int32_t>() + 2, s);
    if (e != hipSuccess) return hip_fail(c, e, "fia_count_related");
    if (total_out) {
      int32_t flags[4] = {0, 0, 0, 0};
      e = hipMemcpyAsync(total_out, offsets + Q, sizeof(int64_t), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipMemcpyAsync(flags, c->flag.ptr, sizeof(flags), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) return hip_fail(c, e, "fia_count_related");
      if (flags[1]) return fail(c, FIA_ERR_INVALID, "query ids out of range [0, num_users) x [0, num_items)");
      if (flags[2])
        return fail(c, FIA_ERR_STATE, "a query's user or item has no Hessian cache: it was not among the "
                                      "queries of the last fia_prepare_for");
    }
    return FIA_OK;
  })
}

int fia_related(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                int32_t* rel_idx, void* stream) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    if (!c->idx.valid) return fail(c, FIA_ERR_STATE, "fia_build_index has not been called");
    if (Q < 0 || Q >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "num_queries out of range");
    if (Q > 0 && (!qu || !qi || !offsets || !rel_idx)) return fail(c, FIA_ERR_INVALID, "null array");
    DeviceGuard g(c->device);
    if (int rc = enter_stream(c, as_stream(stream), "fia_related"); rc != FIA_OK) return rc;
    hipError_t e = fia::write_related(c, Q, qu, qi, offsets, rel_idx, as_stream(stream));
    if (e != hipSuccess) return hip_fail(c, e, "fia_related");
    return FIA_OK;
  })
}

static int query_batch_common(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                              int64_t total_rel, int32_t* rel_idx, double* influence, double* x_out, int K,
                              int64_t* topk_pos, int64_t* topk_idx, double* topk_val, void* stream,
                              const double* x_in) {
  if (!c) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    if (!c->p.valid || !c->idx.valid) return fail(c, FIA_ERR_STATE, "params/index missing");
    if (!c->prepared) return fail(c, FIA_ERR_STATE, "fia_prepare has not been called since params/index changed");
    if (Q < 0 || Q >= (1LL << 31)) return fail(c, FIA_ERR_INVALID, "num_queries out of range");
    if (total_rel < 0) return fail(c, FIA_ERR_INVALID, "total_rel < 0");
    if (K < 0 || K > FIA_MAX_TOPK) return fail(c, FIA_ERR_INVALID, "K must be in [0, FIA_MAX_TOPK]");
    if (Q > 0 && (!qu || !qi || !offsets)) return fail(c, FIA_ERR_INVALID, "null query array");
    if (K > 0 && (!topk_pos || !topk_idx || !topk_val)) return fail(c, FIA_ERR_INVALID, "null top-K output");
    if (Q == 0) return FIA_OK;
    DeviceGuard g(c->device);
    if (int rc = enter_stream(c, as_stream(stream), "fia_query_batch"); rc != FIA_OK) return rc;
    // (small k joins the pending Gram pass right before its solve, after the query scans)
    if (fia::big_supported(c->p.model, c->p.k))
      if (hipError_t es = fia::join_prepare(c, as_stream(stream)); es != hipSuccess) return hip_fail(c, es, "fia_query_batch");
    // chunk descriptors / candidate slots: at most 2 per query + one per chunk of the model's
    // shortest chunk length (NCF k <= 16 runs: kNcfRunChunk; else kRunChunk).  (A tighter bound
    // also keeps ml-1m-ex's top-K merge on its thread-per-query kernel.)
    const int64_t clen = c->p.model == FIA_MODEL_NCF && c->p.k <= 16 ? fia::kNcfRunChunk : fia::kRunChunk;
    const int64_t max_chunks = 2 * Q + total_rel / clen + 1;
    bool unsup = false;
    hipError_t e = fia::query_model(c, Q, qu, qi, offsets, max_chunks, rel_idx, influence, x_out, K, topk_pos,
                                    topk_idx, topk_val, as_stream(stream), unsup, x_in);
    if (unsup) return fail(c, FIA_ERR_UNSUPPORTED, "model/k not supported");
    if (e != hipSuccess) return hip_fail(c, e, "fia_query_batch");
    return FIA_OK;
  })
}

int fia_query_batch(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                    int64_t total_rel, int32_t* rel_idx, double* influence, double* x_out, int K,
                    int64_t* topk_pos, int64_t* topk_idx, double* topk_val, void* stream) {
  return query_batch_common(c, Q, qu, qi, offsets, total_rel, rel_idx, influence, x_out, K, topk_pos, topk_idx,
                            topk_val, stream, nullptr);
}

int fia_query_batch_x(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                      int64_t total_rel, const double* x_in, int32_t* rel_idx, double* influence, int K,
                      int64_t* topk_pos, int64_t* topk_idx, double* topk_val, void* stream) {
  if (!c) return FIA_ERR_INVALID;
  if (Q > 0 && !x_in) return fail(c, FIA_ERR_INVALID, "null x_in");
  return query_batch_common(c, Q, qu, qi, offsets, total_rel, rel_idx, influence, nullptr, K, topk_pos, topk_idx,
                            topk_val, stream, x_in);
}

int fia_set_profiling(fia_ctx* c, int phase_mask) {
  if (!c) return FIA_ERR_INVALID;
  c->profiling = (unsigned)phase_mask & ((1u << FIA_NUM_PHASES) - 1u);
  return FIA_OK;
}

int fia_profile_read(fia_ctx* c, double* ms_sum, int64_t* counts) {
  if (!c || !ms_sum || !counts) return FIA_ERR_INVALID;
  FIA_GUARDED(c, {
    DeviceGuard g(c->device);
    int rc = FIA_OK;
    for (int ph = 0; ph < FIA_NUM_PHASES; ++ph) {
      double sum = 0.0;
      int64_t cnt = 0;
      for (auto& pr : c->events.ev[ph]) {
        float ms = 0.f;
        if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
          sum += ms;
          ++cnt;
        } else {
          rc = fail(c, FIA_ERR_HIP, "event timing failed");
        }
        c->events.pool.push_back(pr.first);
        c->events.pool.push_back(pr.second);
      }
      c->events.ev[ph].clear();
      ms_sum[ph] = sum;
      counts[ph] = cnt;
    }
    return rc;
  })
}

}  // extern "C"
