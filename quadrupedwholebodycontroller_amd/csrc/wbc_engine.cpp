// wbc_engine.cpp — host side of the C-ABI (include/wbc.h): device buffers, stream ordering,
// kernel launches.  Replaces the per-object state of the reference's WholeBodyController
// (include/anymal_wbc/whole_body_controller.hpp:106-166) with batched device buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>

#include "wbc.h"
#include "wbc_anymal_model.h"
#include "wbc_layout.h"


extern "C" hipError_t wbc_launch_step(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_update(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_solve_general(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_solve_stance(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_update_solve(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_stance_step(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_modes(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_reset(double* hist, const uint8_t* mask, int batch, hipStream_t st);
extern "C" hipError_t wbc_launch_qmap(const uint8_t* masks, int batch, int32_t* map, hipStream_t st);
extern "C" hipError_t wbc_preload_resident();
extern "C" hipError_t wbc_launch_resident(const wbc::KernelArgs* a, wbc::ResidentBox* box, const void* pin_in,
                                          void* own_in, int in_words, unsigned long long seq0, unsigned long long idle_ticks,
                                          hipStream_t st);

namespace {
thread_local std::string g_err;

int32_t fail(int32_t code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define WBC_HIP(call)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) return fail(WBC_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)
}  // namespace

struct wbc_engine {
    int32_t batch = 0;
    int32_t device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    wbc_model* d_model = nullptr;
    wbc_params* d_params = nullptr;
    double* d_limg = nullptr;  // the step kernel's LDS image of the model + friction table (wbc_layout.h)
    wbc_params params{};  // host copy, passed by value in the kernel arguments (KernelArgs::pv)
    // owned inputs: one device block [pose | nu | qj | ref | contacts | switching] (so a host cycle
    // is one H2D copy), and the outputs one block [tau | grf | status | iters | x]
    void* d_inblk = nullptr;
    void* d_outblk = nullptr;
    void* h_in = nullptr;   // pinned staging of the same layouts (wbc_cycle, allocated on first use)
    void* h_out = nullptr;
    double* d_pose = nullptr;
    double* d_nu = nullptr;
    double* d_qj = nullptr;
    double* d_ref = nullptr;
    uint8_t* d_contacts = nullptr;
    uint8_t* d_switching = nullptr;
    uint8_t* d_mask = nullptr;
    // contact-mode hypotheses (wbc_set_modes): n_modes > 0 turns the inputs into B / n_modes states
    int32_t n_modes = 0;
    uint8_t* d_modes = nullptr;
    // the update shared by mode_loop hypotheses per wave (KernelArgs::mloop; 1 = one per segment)
    // and the hypotheses' order, chunk by chunk (plan_mode_loop)
    int32_t mode_loop = 1;
    uint8_t mode_order[16] = {};
    // bound (possibly external) inputs
    const double* in_pose = nullptr;
    const double* in_nu = nullptr;
    const double* in_qj = nullptr;
    const double* in_ref = nullptr;
    const uint8_t* in_contacts = nullptr;
    const uint8_t* in_switching = nullptr;
    // state / outputs
    double* d_hist = nullptr;
    double* d_work = nullptr;
    int32_t* d_fb = nullptr;  // elimination fallback counters [2] + list [B] (KernelArgs::fb)
    int32_t parity = 0;       // fallback counter of the next elimination update
    // four-contact rows among the engine's own contact masks (d_contacts, as last copied from the
    // host) and among the mode masks: the stance elimination runs when every QP of a step has
    // mask 15 (known only for the engine's own masks; device-bound masks take the general path)
    int64_t n_stance_own = 0;
    int32_t modes_stance = 0;
    bool elim = false;        // the last update's choice (its solve follows it)
    int32_t elim_parity = 0;  // and its fallback counter
    double* d_tau = nullptr;
    double* d_grf = nullptr;
    double* d_x = nullptr;
    int32_t* d_status = nullptr;
    int32_t* d_iters = nullptr;
    double* d_dbg = nullptr;
    // bound (possibly external) outputs
    double* out_tau = nullptr;
    double* out_grf = nullptr;
    double* out_x = nullptr;
    int32_t* out_status = nullptr;
    int32_t* out_iters = nullptr;
    // the default step's wave map (KernelArgs::qmap): QPs grouped by contact mask, four to a wave.
    // For the engine's own masks it is built on the host whenever they are copied (qmap_waves waves;
    // 0 = every mask equal, no map needed); for device-bound masks wbc_qmap_kernel builds it on the
    // stream before each step
    int32_t* d_qmap = nullptr;
    const int32_t* qmap_dev = nullptr;  // the step's map of the engine's own masks: d_qmap, or m_qmap (zero-copy cycle)
    const uint8_t* m_contacts = nullptr;  // the zero-copy cycle block's masks (device address)
    // a zero-copy cycle ran last: the engine's own input / output blocks (and wave map) are behind the
    // pinned ones until sync_own copies them (before any other call that reads or writes them)
    bool zc_stale = false;
    int32_t* h_qmap = nullptr;  // pinned
    int32_t qmap_waves = 0;
    bool qmap_host = true;  // qmap_waves / d_qmap describe d_contacts (not after a change of modes)
    bool updated = false;
    bool timed = false;    // a WBC_TIMED step has recorded ev0 / ev1
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // device addresses of the pinned cycle buffers (zero-copy cycle: the step reads h_in and writes
    // h_out directly, no copies); null when the batch takes the copy path
    const void* m_in = nullptr;
    void* m_out = nullptr;
    const int32_t* m_qmap = nullptr;
    // the resident control cycle (WBC_RESIDENT): mailbox (pinned, coherent), its stream, whether a
    // resident wave runs and with which step flags, the last command posted, when it last answered
    wbc::ResidentBox* res_box = nullptr;
    wbc::ResidentBox* res_box_dev = nullptr;
    hipStream_t res_stream = nullptr;
    bool res_on = false;
    uint32_t res_flags = 0;
    unsigned long long res_seq = 0;
    std::chrono::steady_clock::time_point res_last{};
};

namespace {
template <class T>
hipError_t dalloc(T** p, size_t n) {
    return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (n ? n : 1));
}

// device input / output block sizes (bytes)
size_t in_block_bytes(size_t B) {
    return B * (WBC_POSE_LEN + WBC_NU_LEN + WBC_NUM_JOINTS + WBC_REF_LEN) * sizeof(double) + 2 * B;
}
size_t out_block_bytes(size_t B) {
    return B * 2 * WBC_NUM_JOINTS * sizeof(double) + 2 * B * sizeof(int32_t) + B * WBC_NV * sizeof(double);
}

// wbc_cycle runs zero-copy up to this batch size (enqueue_cycle)
[[maybe_unused]] constexpr size_t kZeroCopyMaxBatch = 64;

// rows of the input arrays: one per robot, or one per state when mode hypotheses are set
size_t input_rows(const wbc_engine* h) { return (size_t)(h->n_modes ? h->batch / h->n_modes : h->batch); }

wbc::KernelArgs make_args(wbc_engine* h, uint32_t flags) {
    wbc::KernelArgs a;
    a.model = h->d_model;
    a.params = h->d_params;
    a.limg = h->d_limg;
    a.pv = h->params;
    a.base_pose = h->in_pose;
    a.nu = h->in_nu;
    a.qj = h->in_qj;
    a.ref = h->in_ref;
    a.contacts = h->in_contacts;
    a.switching = h->in_switching;
    a.hist = h->d_hist;
    a.work = h->d_work;
    a.tau = h->out_tau;
    a.grf = h->out_grf;
    a.x = (flags & WBC_NO_X) ? nullptr : h->out_x;
    a.status = h->out_status;
    a.iters = h->out_iters;
    a.dbg = h->d_dbg;
    a.batch = h->batch;
    a.stateful = (flags & WBC_STATELESS) ? 0 : 1;
    a.debug = (flags & WBC_DEBUG) ? 1 : 0;
    a.cold = (flags & WBC_COLD) ? 1 : 0;
    a.modes = 0;
    a.mode_masks = h->d_modes;
    a.elim = 0;
    a.parity = 0;
    a.fb = h->d_fb;
    a.fb_cap = h->batch;
    a.qmap = nullptr;
    a.nwaves = (h->batch + wbc::QMAP_SEG - 1) / wbc::QMAP_SEG;
    a.mloop = 0;
    std::memset(a.mode_order, 0, sizeof(a.mode_order));
    return a;
}

// Host wave map of the engine's own contact masks (copied on the stream; the callers synchronize
// before the host buffer is reused)
hipError_t upload_qmap(wbc_engine* h, const uint8_t* masks) {
    h->qmap_waves = wbc::qmap_build(masks, h->batch, h->h_qmap);
    h->qmap_host = true;
    if (!h->qmap_waves) return hipSuccess;
    return hipMemcpyAsync(h->d_qmap, h->h_qmap, (size_t)h->qmap_waves * wbc::QMAP_SEG * sizeof(int32_t),
                          hipMemcpyHostToDevice, h->stream);
}

// wait for every launch the engine queued so far: a stream synchronize of the bound stream (its
// own, or the caller's, which must still be alive: include/wbc.h, wbc_set_stream).  No event is
// recorded per launch: an event packet between two steps costs ~3 us of the ~36 us step (measured
// on MI355X, 103.5 -> 112.3 M solves/s on the headline config without it).
hipError_t drain(wbc_engine* h) { return h->stream ? hipStreamSynchronize(h->stream) : hipSuccess; }

// Mode hypotheses per wave and their order (wbc_layout.h mode_loop_plan) for this engine's batch
// and device: every SIMD (4 per CU) should get a wave.  WBC_MODES_M (a divisor of K) overrides M
// (A/B runs, tests).
void plan_mode_loop(wbc_engine* h, const uint8_t* modes, int32_t K) {
    const int64_t groups = (h->batch / K + 3) / 4;
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus <= 0) cus = 256;
    const char* e = std::getenv("WBC_MODES_M");
    h->mode_loop = wbc::mode_loop_plan(modes, K, groups, 4LL * cus, e ? std::atoi(e) : 0, h->mode_order);
}

int64_t count_stance(const uint8_t* masks, size_t n) {
    int64_t c = 0;
    for (size_t i = 0; i < n; ++i) c += (masks[i] & 15) == 15;
    return c;
}

// The resident cycle's mailbox (pinned, coherent) and stream; at wbc_create for B <= 4 (a few ms that
// would otherwise land on the first resident cycle)
hipError_t resident_alloc(wbc_engine* h) {
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, sizeof(wbc::ResidentBox), hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    std::memset(p, 0, sizeof(wbc::ResidentBox));
    h->res_box = static_cast<wbc::ResidentBox*>(p);
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, p, 0);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->res_stream, hipStreamNonBlocking);
    h->res_box_dev = static_cast<wbc::ResidentBox*>(d);
    h->res_seq = 0;
    return e;
}

// At most one resident wave runs per process: a resident kernel holds its hardware queue
// between cycles, and streams share the GPU_MAX_HW_QUEUES queues, so another engine's work could wait
// behind it until its idle exit.  g_res_owner is the engine whose wave runs; every start and stop of a
// resident wave holds g_res_mu, and every other engine's call that launches work stops that wave first
// (sync_own).  Streams of other libraries (torch) are not covered: INTEGRATION.md states the limit.
std::recursive_mutex g_res_mu;
wbc_engine* g_res_owner = nullptr;

// The resident cycle's wave (WBC_RESIDENT) ends: WBC_RESIDENT_STOP posted, then its stream drained
// (it may have ended by itself after its idle time: then it is idle at once).  Bounded: a wave that
// does not end within kResidentStopWait (stuck inside a step) is reported, not waited for forever.
constexpr auto kResidentStopWait = std::chrono::seconds(2);
hipError_t resident_stop(wbc_engine* h) {
    std::lock_guard<std::recursive_mutex> lk(g_res_mu);
    if (!h->res_on) return hipSuccess;
    h->res_on = false;
    if (g_res_owner == h) g_res_owner = nullptr;
    __atomic_store_n(&h->res_box->cmd, wbc::WBC_RESIDENT_STOP, __ATOMIC_RELEASE);
    const auto deadline = std::chrono::steady_clock::now() + kResidentStopWait;
    hipError_t e;
    while ((e = hipStreamQuery(h->res_stream)) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() > deadline) return hipErrorLaunchTimeOut;
        std::this_thread::yield();
    }
    __atomic_store_n(&h->res_box->cmd, h->res_seq, __ATOMIC_RELEASE);  // the next wave starts from res_seq
    return e;
}

// Another engine's resident wave on this engine's device, stopped before this engine launches work.
hipError_t stop_foreign_resident(wbc_engine* h) {
    std::lock_guard<std::recursive_mutex> lk(g_res_mu);
    if (!g_res_owner || g_res_owner == h || g_res_owner->device != h->device) return hipSuccess;
    return resident_stop(g_res_owner);
}

// After a zero-copy wbc_cycle the cycle's inputs, outputs and wave map live in the pinned blocks;
// copy them into the engine's own device buffers, so every other call sees the state a copying
// cycle leaves (synchronous: the pinned blocks are rewritten by the next cycle).  A resident cycle
// wave is stopped first, this engine's or another engine's on the same device (every other call goes
// through here).
hipError_t sync_own(wbc_engine* h) {
    {
        hipError_t e = resident_stop(h);
        if (e == hipSuccess) e = stop_foreign_resident(h);
        if (e != hipSuccess) return e;
    }
    if (!h->zc_stale) return hipSuccess;
    const size_t B = (size_t)h->batch;
    hipError_t e = hipSetDevice(h->device);
    if (e == hipSuccess) e = hipMemcpyAsync(h->d_inblk, h->h_in, in_block_bytes(B), hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(h->d_outblk, h->h_out, out_block_bytes(B), hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess && h->qmap_waves)
        e = hipMemcpyAsync(h->d_qmap, h->h_qmap, (size_t)h->qmap_waves * wbc::QMAP_SEG * sizeof(int32_t),
                           hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) h->zc_stale = false;
    return e;
}

// Stance elimination for this update: on when every QP has mask 15 (a mixed batch would pay the
// elimination in the update kernel's mixed waves and a second solve kernel's latency; measured
// slower, profiles/r02/k), which the host knows for its own contact masks and for mode masks.
void begin_update(wbc_engine* h, wbc::KernelArgs& a) {
    bool all = false;
    if (h->n_modes) all = h->modes_stance == h->n_modes;
    else if (h->in_contacts == h->d_contacts) all = h->n_stance_own == h->batch;
    h->elim = all;
    // the fallback counters alternate between elimination updates only: the update with parity p
    // fills fb[p] and clears fb[p ^ 1], which only the next elimination update uses (an update
    // without the elimination neither fills nor clears a list, so it must not move the parity)
    h->elim_parity = h->parity;
    if (h->elim) h->parity ^= 1;
    a.elim = h->elim ? 1 : 0;
    a.parity = h->elim_parity;
}

// The default step (wbc_update_solve_kernel: every QP reduced to 12 variables and solved in the
// update wave) solves its own fallbacks in the wave that found them (no list), so it
// leaves the fallback list and its parity to the split path's elimination updates.  Its waves each
// hold QPs of one contact mask: the wave map (the engine's own masks: built when they were copied;
// device-bound masks: built on the stream now under WBC_GROUP), or under mode hypotheses the
// arithmetic map.
hipError_t begin_step16(wbc_engine* h, wbc::KernelArgs& a, uint32_t flags) {
    a.elim = 1;
    h->elim = false;  // a later wbc_solve needs its own wbc_update
    if (a.modes) {
        const int S = h->batch / a.modes;
        a.nwaves = ((S + wbc::QMAP_SEG - 1) / wbc::QMAP_SEG) * a.modes;
        return hipSuccess;
    }
    if ((h->in_contacts == h->d_contacts || (h->m_contacts && h->in_contacts == h->m_contacts)) && h->qmap_host) {
#ifndef WBC_NO_QMAP  // (A/B builds only: the unmapped step)
        if (h->qmap_waves) {
            a.qmap = h->qmap_dev;
            a.nwaves = h->qmap_waves;
        }
#endif
        return hipSuccess;
    }
    // device-bound masks: the map is built on the stream when the caller asks for it (WBC_GROUP);
    // otherwise waves take four consecutive QPs (same results; a wave of mixed masks costs more)
    if (!(flags & WBC_GROUP)) return hipSuccess;
    a.qmap = h->d_qmap;
    a.nwaves = wbc::qmap_capacity(h->batch) / wbc::QMAP_SEG;
    return wbc_launch_qmap(h->in_contacts, h->batch, h->d_qmap, h->stream);
}

// The default step's QPs are all stance QPs of the stance form: stateless, the engine's own masks
// (copied by the host, counted at copy time), every one 15, no map and no mode hypotheses.
bool step_all_stance(const wbc_engine* h, const wbc::KernelArgs& a) {
#ifdef WBC_NO_STANCE_TU  // (A/B builds only: the mixed-form kernel for every step)
    return false;
#else
    const bool own = h->in_contacts == h->d_contacts || (h->m_contacts && h->in_contacts == h->m_contacts);
    return own && h->qmap_host && h->n_stance_own == h->batch && !a.stateful && !a.modes && !a.qmap;
#endif
}

hipError_t launch_solves(wbc_engine* h, wbc::KernelArgs& a) {
    a.elim = h->elim ? 1 : 0;
    a.parity = h->elim_parity;
    return h->elim ? wbc_launch_solve_stance(&a, h->stream) : wbc_launch_solve_general(&a, h->stream);
}
}  // namespace

extern "C" {

int32_t wbc_default_params(wbc_params* p) {
    if (!p) return fail(WBC_ERR_ARG, "null params");
    std::memset(p, 0, sizeof(*p));
    p->friction = 1.0;       // params_controller.yaml:2
    p->loop_rate = 400.0;    // :3
    p->max_torque = 80.0;    // :4
    p->kp = 6000.0;          // :5
    p->kp_z = 10000.0;       // :6
    p->kd = 1800.0;          // :7
    p->ki = 0.0;             // :8
    p->kp_swing = 250.0;     // :9
    p->kd_swing = 20.0;      // :10
    p->slack_weight = 1000.0;  // :11
    const double pose[6] = {0.0, 0.0, 0.50, 0.0, 0.0, 0.0};  // :12
    std::memcpy(p->initial_reference_pose, pose, sizeof(pose));
    p->gravity = 9.81;       // hpp:30
    p->max_wsr = 100;        // cpp:517
    return WBC_OK;
}

int32_t wbc_anymal_model(wbc_model* m) {
    if (!m) return fail(WBC_ERR_ARG, "null model");
    *m = WBC_ANYMAL_MODEL;
    return WBC_OK;
}

int32_t wbc_create(const wbc_model* model, const wbc_params* params, int32_t batch, int32_t device, wbc_engine** out) {
    if (!out || batch <= 0) return fail(WBC_ERR_ARG, "wbc_create: bad arguments");
    if (batch > wbc::QMAP_MAX_BATCH) return fail(WBC_ERR_ARG, "wbc_create: batch above 2^27 - 1 (the wave map's index range)");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(WBC_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(WBC_ERR_ARG, "wbc_create: bad device index");
    WBC_HIP(hipSetDevice(device));
    wbc_engine* h = new (std::nothrow) wbc_engine();
    if (!h) return fail(WBC_ERR_ARG, "out of host memory");
    h->batch = batch;
    h->device = device;
    wbc_model m = model ? *model : WBC_ANYMAL_MODEL;
    wbc_params p;
    if (params) p = *params;
    else wbc_default_params(&p);
    if (p.loop_rate <= 0.0 || p.max_wsr <= 0) {
        delete h;
        return fail(WBC_ERR_ARG, "wbc_create: invalid params");
    }
    h->params = p;
    const size_t B = (size_t)batch;
#define ALLOC(ptr, n)                                             \
    if (dalloc(&h->ptr, (n)) != hipSuccess) {                     \
        wbc_destroy(h);                                           \
        return fail(WBC_ERR_HIP, "hipMalloc failed: " #ptr);      \
    }
    ALLOC(d_model, 1);
    ALLOC(d_params, 1);
    ALLOC(d_limg, wbc::LIMG_LEN);
    // (the input block in whole 8-byte words: the resident cycle copies it by words)
    if (hipMalloc(&h->d_inblk, (in_block_bytes(B) + 7) / 8 * 8) != hipSuccess ||
        hipMalloc(&h->d_outblk, out_block_bytes(B)) != hipSuccess) {
        wbc_destroy(h);
        return fail(WBC_ERR_HIP, "hipMalloc failed: input/output blocks");
    }
    {
        double* in = static_cast<double*>(h->d_inblk);
        h->d_pose = in;
        h->d_nu = h->d_pose + B * WBC_POSE_LEN;
        h->d_qj = h->d_nu + B * WBC_NU_LEN;
        h->d_ref = h->d_qj + B * WBC_NUM_JOINTS;
        h->d_contacts = reinterpret_cast<uint8_t*>(h->d_ref + B * WBC_REF_LEN);
        h->d_switching = h->d_contacts + B;
        double* out = static_cast<double*>(h->d_outblk);
        h->d_tau = out;
        h->d_grf = h->d_tau + B * WBC_NUM_JOINTS;
        h->d_status = reinterpret_cast<int32_t*>(h->d_grf + B * WBC_NUM_JOINTS);
        h->d_iters = h->d_status + B;
        h->d_x = reinterpret_cast<double*>(h->d_iters + B);  // status + iters = 8 B per robot: aligned
    }
    ALLOC(d_mask, B);
    ALLOC(d_modes, WBC_MAX_MODES);
    ALLOC(d_hist, B * wbc::HIST_LEN);
    ALLOC(d_work, B * wbc::WORK_LEN);
    ALLOC(d_fb, 2 + B);
    ALLOC(d_dbg, B * WBC_DBG_LEN);
    ALLOC(d_qmap, wbc::qmap_capacity(batch) + wbc::qmap_scratch(batch));  // + the device builder's scratch
#undef ALLOC
    if (hipHostMalloc(&h->h_qmap, sizeof(int32_t) * wbc::qmap_capacity(batch), hipHostMallocMapped) != hipSuccess) {
        wbc_destroy(h);
        return fail(WBC_ERR_HIP, "hipHostMalloc failed: wave map");
    }
    h->qmap_dev = h->d_qmap;
    if (B <= (size_t)wbc::QMAP_SEG) {  // the resident cycle's code and mailbox, made ready now
        (void)wbc_preload_resident();
        if (resident_alloc(h) != hipSuccess) {
            wbc_destroy(h);
            return fail(WBC_ERR_HIP, "resident cycle mailbox / stream");
        }
    }
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
        wbc_destroy(h);
        return fail(WBC_ERR_HIP, "stream/event creation failed");
    }
    h->stream = h->own_stream;
    h->n_stance_own = B;  // d_contacts starts as all-stance (15), below
    h->in_pose = h->d_pose;
    h->in_nu = h->d_nu;
    h->in_qj = h->d_qj;
    h->in_ref = h->d_ref;
    h->in_contacts = h->d_contacts;
    h->in_switching = h->d_switching;
    h->out_tau = h->d_tau;
    h->out_grf = h->d_grf;
    h->out_x = h->d_x;
    h->out_status = h->d_status;
    h->out_iters = h->d_iters;
    hipStream_t st = h->stream;
    wbc::LdsImage limg;
    wbc::build_lds_image(m, p.friction, limg);
    if (hipMemcpyAsync(h->d_model, &m, sizeof(m), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(h->d_params, &p, sizeof(p), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(h->d_limg, &limg, sizeof(limg), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemsetAsync(h->d_pose, 0, B * WBC_POSE_LEN * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_nu, 0, B * WBC_NU_LEN * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_qj, 0, B * WBC_NUM_JOINTS * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_ref, 0, B * WBC_REF_LEN * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_contacts, 15, B, st) != hipSuccess ||
        hipMemsetAsync(h->d_switching, 0, B, st) != hipSuccess ||
        hipMemsetAsync(h->d_status, 0, B * sizeof(int32_t), st) != hipSuccess ||
        hipMemsetAsync(h->d_iters, 0, B * sizeof(int32_t), st) != hipSuccess ||
        hipMemsetAsync(h->d_tau, 0, B * WBC_NUM_JOINTS * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_grf, 0, B * WBC_NUM_JOINTS * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_x, 0, B * WBC_NV * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_dbg, 0, B * WBC_DBG_LEN * sizeof(double), st) != hipSuccess ||
        hipMemsetAsync(h->d_fb, 0, (2 + B) * sizeof(int32_t), st) != hipSuccess ||
        wbc_launch_reset(h->d_hist, nullptr, batch, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        wbc_destroy(h);
        return fail(WBC_ERR_HIP, "wbc_create: initialisation failed");
    }
    *out = h;
    return WBC_OK;
}

int32_t wbc_destroy(wbc_engine* h) {
    if (!h) return WBC_OK;
    (void)hipSetDevice(h->device);
    // drain the engine's in-flight work before freeing (the bound stream; never the whole device,
    // which would also wait for other engines' and the caller's unrelated work)
    (void)drain(h);
    {
        std::lock_guard<std::recursive_mutex> lk(g_res_mu);
        (void)resident_stop(h);
        if (g_res_owner == h) g_res_owner = nullptr;  // never left pointing at a freed engine
    }
    if (h->res_box) (void)hipHostFree(h->res_box);
    if (h->res_stream) (void)hipStreamDestroy(h->res_stream);
    void* ptrs[] = {h->d_model, h->d_params, h->d_limg, h->d_inblk, h->d_outblk, h->d_mask, h->d_modes, h->d_hist, h->d_work,
                    h->d_fb, h->d_dbg, h->d_qmap};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (h->h_in) (void)hipHostFree(h->h_in);
    if (h->h_out) (void)hipHostFree(h->h_out);
    if (h->h_qmap) (void)hipHostFree(h->h_qmap);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return WBC_OK;
}

int32_t wbc_batch(const wbc_engine* h) { return h ? h->batch : 0; }

int32_t wbc_set_stream(wbc_engine* h, void* stream) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    const hipStream_t next = stream ? reinterpret_cast<hipStream_t>(stream) : h->own_stream;
    if (next != h->stream) {
        // work already queued on the old stream still reads the engine's buffers: let it finish
        // before any call on the new stream can overwrite them
        WBC_HIP(hipSetDevice(h->device));
        WBC_HIP(drain(h));
    }
    h->stream = next;
    return WBC_OK;
}

int32_t wbc_set_state(wbc_engine* h, const double* base_pose, const double* nu, const double* qj) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    WBC_HIP(hipSetDevice(h->device));
    const size_t B = input_rows(h);
    if (base_pose) { WBC_HIP(hipMemcpyAsync(h->d_pose, base_pose, B * WBC_POSE_LEN * sizeof(double), hipMemcpyHostToDevice, h->stream)); h->in_pose = h->d_pose; }
    if (nu) { WBC_HIP(hipMemcpyAsync(h->d_nu, nu, B * WBC_NU_LEN * sizeof(double), hipMemcpyHostToDevice, h->stream)); h->in_nu = h->d_nu; }
    if (qj) { WBC_HIP(hipMemcpyAsync(h->d_qj, qj, B * WBC_NUM_JOINTS * sizeof(double), hipMemcpyHostToDevice, h->stream)); h->in_qj = h->d_qj; }
    WBC_HIP(hipStreamSynchronize(h->stream));  // host buffers may be reused by the caller
    return WBC_OK;
}

int32_t wbc_set_reference(wbc_engine* h, const double* ref, const uint8_t* contacts, const uint8_t* switching) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    WBC_HIP(hipSetDevice(h->device));
    const size_t B = input_rows(h);
    if (ref) { WBC_HIP(hipMemcpyAsync(h->d_ref, ref, B * WBC_REF_LEN * sizeof(double), hipMemcpyHostToDevice, h->stream)); h->in_ref = h->d_ref; }
    if (contacts) {
        WBC_HIP(hipMemcpyAsync(h->d_contacts, contacts, B, hipMemcpyHostToDevice, h->stream));
        h->in_contacts = h->d_contacts;
        h->n_stance_own = count_stance(contacts, B);
        // the wave map of these masks (rows = QPs; under mode hypotheses contacts[] is not read)
        if (!h->n_modes) WBC_HIP(upload_qmap(h, contacts));
    }
    if (switching) { WBC_HIP(hipMemcpyAsync(h->d_switching, switching, B, hipMemcpyHostToDevice, h->stream)); h->in_switching = h->d_switching; }
    WBC_HIP(hipStreamSynchronize(h->stream));
    return WBC_OK;
}

int32_t wbc_bind_device_inputs(wbc_engine* h, const double* d_base_pose, const double* d_nu, const double* d_qj,
                               const double* d_ref, const uint8_t* d_contacts, const uint8_t* d_switching) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    h->in_pose = d_base_pose ? d_base_pose : h->d_pose;
    h->in_nu = d_nu ? d_nu : h->d_nu;
    h->in_qj = d_qj ? d_qj : h->d_qj;
    h->in_ref = d_ref ? d_ref : h->d_ref;
    h->in_contacts = d_contacts ? d_contacts : h->d_contacts;
    h->in_switching = d_switching ? d_switching : h->d_switching;
    return WBC_OK;
}

int32_t wbc_bind_device_outputs(wbc_engine* h, double* d_tau, double* d_grf, double* d_x, int32_t* d_status,
                                int32_t* d_iters) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    h->out_tau = d_tau ? d_tau : h->d_tau;
    h->out_grf = d_grf ? d_grf : h->d_grf;
    h->out_x = d_x ? d_x : h->d_x;
    h->out_status = d_status ? d_status : h->d_status;
    h->out_iters = d_iters ? d_iters : h->d_iters;
    return WBC_OK;
}

int32_t wbc_reset(wbc_engine* h, const uint8_t* mask) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    WBC_HIP(hipSetDevice(h->device));
    const uint8_t* dm = nullptr;
    if (mask) {
        WBC_HIP(hipMemcpyAsync(h->d_mask, mask, (size_t)h->batch, hipMemcpyHostToDevice, h->stream));
        dm = h->d_mask;
    }
    WBC_HIP(wbc_launch_reset(h->d_hist, dm, h->batch, h->stream));
    WBC_HIP(hipStreamSynchronize(h->stream));
    h->updated = false;
    return WBC_OK;
}

int32_t wbc_update(wbc_engine* h, uint32_t flags) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    if (h->n_modes) return fail(WBC_ERR_STATE, "wbc_update: mode hypotheses are set (use wbc_step_modes, or wbc_set_modes(h, 0, NULL))");
    WBC_HIP(hipSetDevice(h->device));
    wbc::KernelArgs a = make_args(h, flags);
    begin_update(h, a);
    WBC_HIP(wbc_launch_update(&a, h->stream));
    h->updated = true;
    return WBC_OK;
}

int32_t wbc_solve(wbc_engine* h, uint32_t flags) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    if (h->n_modes) return fail(WBC_ERR_STATE, "wbc_solve: mode hypotheses are set (use wbc_step_modes, or wbc_set_modes(h, 0, NULL))");
    if (!h->updated) return fail(WBC_ERR_STATE, "wbc_solve before wbc_update");
    WBC_HIP(hipSetDevice(h->device));
    wbc::KernelArgs a = make_args(h, flags);
    WBC_HIP(launch_solves(h, a));
    return WBC_OK;  // the assembled problem stays valid: solving it again gives the same result
}

int32_t wbc_step(wbc_engine* h, uint32_t flags) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    if (h->n_modes) return fail(WBC_ERR_STATE, "wbc_step: mode hypotheses are set (use wbc_step_modes, or wbc_set_modes(h, 0, NULL))");
    WBC_HIP(hipSetDevice(h->device));
    wbc::KernelArgs a = make_args(h, flags);
    const bool timed = (flags & WBC_TIMED) != 0;  // event packets cost a few us between kernels
    if (timed) WBC_HIP(hipEventRecord(h->ev0, h->stream));
    if (flags & WBC_SPLIT) {
        // the split kernels: update (records to HBM), then the general / stance solve kernels
        begin_update(h, a);
        WBC_HIP(wbc_launch_update(&a, h->stream));
        WBC_HIP(launch_solves(h, a));
    } else if (flags & WBC_FUSED) {
        WBC_HIP(wbc_launch_step(&a, h->stream));  // one robot per wave, the general method
    } else {
        // default: one kernel, every QP reduced to 12 variables and solved in the update wave; a
        // stateless step whose masks the host knows to be all 15 (no map then) runs the stance-only
        // instance, scheduled for it alone (wbc_kernel_stance.hip)
        WBC_HIP(begin_step16(h, a, flags));
        if (step_all_stance(h, a)) WBC_HIP(wbc_launch_stance_step(&a, h->stream));
        else WBC_HIP(wbc_launch_update_solve(&a, h->stream));
    }
    if (timed) {
        WBC_HIP(hipEventRecord(h->ev1, h->stream));
        h->timed = true;
    }
    h->updated = false;
    return WBC_OK;
}

int32_t wbc_set_modes(wbc_engine* h, int32_t n_modes, const uint8_t* modes) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    // contacts[] copied while modes were set hold S rows only: the engine's own masks get their
    // wave map on the device from here on, until the next wbc_set_reference / wbc_cycle with masks
    h->qmap_host = false;
    if (n_modes == 0) {
        h->n_modes = 0;
        return WBC_OK;
    }
    if (n_modes < 0 || n_modes > WBC_MAX_MODES || !modes || h->batch % n_modes != 0)
        return fail(WBC_ERR_ARG, "wbc_set_modes: need 1 <= n_modes <= WBC_MAX_MODES dividing the batch, and masks");
    for (int32_t k = 0; k < n_modes; ++k)
        if (modes[k] > 15) return fail(WBC_ERR_ARG, "wbc_set_modes: contact masks are 4-bit");
    WBC_HIP(hipSetDevice(h->device));
    WBC_HIP(hipMemcpyAsync(h->d_modes, modes, (size_t)n_modes, hipMemcpyHostToDevice, h->stream));
    WBC_HIP(hipStreamSynchronize(h->stream));
    h->n_modes = n_modes;
    h->modes_stance = (int32_t)count_stance(modes, (size_t)n_modes);
    plan_mode_loop(h, modes, n_modes);
    return WBC_OK;
}

int32_t wbc_step_modes(wbc_engine* h, uint32_t flags) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    if (!h->n_modes) return fail(WBC_ERR_STATE, "wbc_step_modes: no mode hypotheses set (wbc_set_modes)");
    if (!(flags & WBC_STATELESS)) return fail(WBC_ERR_ARG, "wbc_step_modes: hypotheses are cold steps (WBC_STATELESS)");
    if (flags & WBC_DEBUG) return fail(WBC_ERR_ARG, "wbc_step_modes: no debug records for hypotheses");
    WBC_HIP(hipSetDevice(h->device));
    wbc::KernelArgs a = make_args(h, flags);
    a.modes = h->n_modes;
    const bool timed = (flags & WBC_TIMED) != 0;
    if (timed) WBC_HIP(hipEventRecord(h->ev0, h->stream));
    if (flags & WBC_SPLIT) {
        // split form: the update once per state (problem records to HBM), the general / stance
        // solve kernels once per hypothesis
        begin_update(h, a);
        wbc::KernelArgs au = a;
        au.batch = h->batch / h->n_modes;
        WBC_HIP(wbc_launch_update(&au, h->stream));
        WBC_HIP(launch_solves(h, a));
    } else if (h->mode_loop > 1) {
        // default, many states: one update per state and wave, then mode_loop hypotheses in turn
        a.elim = 1;
        h->elim = false;
        a.mloop = h->mode_loop;
        std::memcpy(a.mode_order, h->mode_order, sizeof(a.mode_order));
        const int64_t S = h->batch / h->n_modes;
        a.nwaves = (int32_t)(((S + wbc::QMAP_SEG - 1) / wbc::QMAP_SEG) * (h->n_modes / h->mode_loop));
        WBC_HIP(wbc_launch_modes(&a, h->stream));
    } else {
        // default: each hypothesis reduced and solved in its own 16-lane segment
        WBC_HIP(begin_step16(h, a, flags));
        WBC_HIP(wbc_launch_update_solve(&a, h->stream));
    }
    if (timed) {
        WBC_HIP(hipEventRecord(h->ev1, h->stream));
        h->timed = true;
    }
    h->updated = false;
    return WBC_OK;
}

}  // extern "C"
namespace {
// One cycle's device work on the engine stream, from the packed pinned inputs (h_in) to the packed
// pinned outputs (h_out): one H2D copy, the wave map's copy when the masks differ, the step on the
// engine's own input and output buffers (caller bindings are restored afterwards), one D2H copy
// (x, last in the block, only without WBC_NO_X).
int32_t enqueue_cycle(wbc_engine* h, uint32_t flags) {
    h->zc_stale = false;  // this cycle's blocks replace whatever was pending
    const size_t B = (size_t)h->batch;
    const size_t inb = in_block_bytes(B), outb = out_block_bytes(B), xb = B * WBC_NV * sizeof(double);
    const bool zc = h->m_in != nullptr;
    if (!zc) {
        WBC_HIP(hipMemcpyAsync(h->d_inblk, h->h_in, inb, hipMemcpyHostToDevice, h->stream));
        if (h->qmap_waves)
            WBC_HIP(hipMemcpyAsync(h->d_qmap, h->h_qmap, (size_t)h->qmap_waves * wbc::QMAP_SEG * sizeof(int32_t),
                                   hipMemcpyHostToDevice, h->stream));
    }
    // the step's input and output block: the engine's device buffers, or (zero-copy) the pinned
    // host buffers through their device addresses, in the same layouts
    const double* ib = zc ? static_cast<const double*>(h->m_in) : static_cast<const double*>(h->d_inblk);
    double* ob = zc ? static_cast<double*>(h->m_out) : static_cast<double*>(h->d_outblk);
    const double* const ip = h->in_pose; const double* const in = h->in_nu; const double* const iq = h->in_qj;
    const double* const ir = h->in_ref; const uint8_t* const ic = h->in_contacts; const uint8_t* const is = h->in_switching;
    h->in_pose = ib;
    h->in_nu = ib + B * WBC_POSE_LEN;
    h->in_qj = h->in_nu + B * WBC_NU_LEN;
    h->in_ref = h->in_qj + B * WBC_NUM_JOINTS;
    h->in_contacts = reinterpret_cast<const uint8_t*>(h->in_ref + B * WBC_REF_LEN);
    h->in_switching = h->in_contacts + B;
    double* const bt = h->out_tau; double* const bg = h->out_grf; double* const bx = h->out_x;
    int32_t* const bs = h->out_status; int32_t* const bi = h->out_iters;
    h->out_tau = ob;
    h->out_grf = ob + B * WBC_NUM_JOINTS;
    h->out_status = reinterpret_cast<int32_t*>(h->out_grf + B * WBC_NUM_JOINTS);
    h->out_iters = h->out_status + B;
    h->out_x = reinterpret_cast<double*>(h->out_iters + B);
    const int32_t* const qm = h->qmap_dev;
    if (zc) h->qmap_dev = h->m_qmap;
    const int32_t rc = wbc_step(h, flags);
    h->qmap_dev = qm;
    h->out_tau = bt; h->out_grf = bg; h->out_x = bx; h->out_status = bs; h->out_iters = bi;
    h->in_pose = ip; h->in_nu = in; h->in_qj = iq; h->in_ref = ir; h->in_contacts = ic; h->in_switching = is;
    // zero-copy: the pinned blocks hold this cycle's inputs (and map) whether or not the step ran, and
    // the host-side mask count / map already describe them, so the own buffers follow them at the next
    // sync_own in either case (on a failed step too, so d_contacts never lags n_stance_own / h_qmap)
    h->zc_stale = zc;
    if (rc != WBC_OK) return rc;
    if (!zc)
        WBC_HIP(hipMemcpyAsync(h->h_out, h->d_outblk, (flags & WBC_NO_X) ? outb - xb : outb, hipMemcpyDeviceToHost,
                               h->stream));
    return WBC_OK;
}
// The resident cycle (WBC_RESIDENT, B <= 4): start the wave if it is not running (or runs with other
// flags, or may have ended by itself: no answer for 40 ms, against its 100 ms idle limit), post the
// cycle, wait for its answer (bounded), and leave the outputs in the pinned output block.
constexpr unsigned long long kResidentIdleTicks = 10000000ull;  // 100 ms of the 100 MHz constant clock
constexpr auto kResidentRestart = std::chrono::milliseconds(40);
constexpr auto kResidentAnswer = std::chrono::seconds(2);
int32_t resident_cycle(wbc_engine* h, uint32_t flags) {
    using clk = std::chrono::steady_clock;
    std::lock_guard<std::recursive_mutex> lk(g_res_mu);
    // wbc_cycle has written this cycle's pinned inputs and the host's mask count / map: the own
    // buffers follow them at the next sync_own whether or not the cycle below succeeds (as
    // enqueue_cycle does on every path), so d_contacts never lags n_stance_own / h_qmap
    h->zc_stale = true;
    const size_t B = (size_t)h->batch;
    WBC_HIP(stop_foreign_resident(h));
    if (h->res_on && (h->res_flags != flags || clk::now() - h->res_last > kResidentRestart)) WBC_HIP(resident_stop(h));
    const auto launch = [&](unsigned long long seq0) -> hipError_t {
        // work queued on the engine stream (a reset, copies) completes before the wave reads the history
        hipError_t e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return e;
        // the step reads the engine's own device input block (the wave copies the pinned block into it
        // every cycle) and writes the pinned output block through its device address
        const double* ib = static_cast<const double*>(h->d_inblk);
        double* ob = static_cast<double*>(h->m_out);
        wbc::KernelArgs a = make_args(h, flags);
        a.base_pose = ib;
        a.nu = ib + B * WBC_POSE_LEN;
        a.qj = a.nu + B * WBC_NU_LEN;
        a.ref = a.qj + B * WBC_NUM_JOINTS;
        a.contacts = reinterpret_cast<const uint8_t*>(a.ref + B * WBC_REF_LEN);
        a.switching = a.contacts + B;
        a.tau = ob;
        a.grf = ob + B * WBC_NUM_JOINTS;
        a.status = reinterpret_cast<int32_t*>(a.grf + B * WBC_NUM_JOINTS);
        a.iters = a.status + B;
        a.x = (flags & WBC_NO_X) ? nullptr : reinterpret_cast<double*>(a.iters + B);
        a.elim = 1;  // as begin_step16: the default step
        a.qmap = nullptr;  // one wave: its robots in batch order
        a.nwaves = 1;
        __atomic_store_n(&h->res_box->exited, 0ull, __ATOMIC_RELEASE);
        const int words = (int)((in_block_bytes(B) + 7) / 8);
        e = wbc_launch_resident(&a, h->res_box_dev, h->m_in, h->d_inblk, words, seq0, kResidentIdleTicks, h->res_stream);
        if (e != hipSuccess) return e;
        h->res_on = true;
        h->res_flags = flags;
        g_res_owner = h;
        return hipSuccess;
    };
    if (!h->res_on) {
        if (!h->res_box) WBC_HIP(resident_alloc(h));
        __atomic_store_n(&h->res_box->cmd, h->res_seq, __ATOMIC_RELEASE);
        WBC_HIP(launch(h->res_seq));
    }
    const unsigned long long seq = ++h->res_seq;
    __atomic_store_n(&h->res_box->cmd, seq, __ATOMIC_RELEASE);  // the inputs (pinned) are written before
    const auto deadline = clk::now() + kResidentAnswer;
    bool relaunched = false;
    while (__atomic_load_n(&h->res_box->done, __ATOMIC_ACQUIRE) != seq) {
        if (!relaunched && __atomic_load_n(&h->res_box->exited, __ATOMIC_ACQUIRE) == 1ull &&
            __atomic_load_n(&h->res_box->done, __ATOMIC_ACQUIRE) != seq) {
            // the wave reached its idle limit just before this cycle was posted (the host thread
            // stalled past kResidentRestart's margin): start a new one from the previous cycle; it
            // picks the posted cycle up
            h->res_on = false;
            if (g_res_owner == h) g_res_owner = nullptr;  // (launch sets it again on success)
            WBC_HIP(launch(seq - 1));
            relaunched = true;
        }
        if (clk::now() > deadline) {
            (void)resident_stop(h);
            return fail(WBC_ERR_HIP, "wbc_cycle: the resident step did not answer");
        }
        __builtin_ia32_pause();
    }
    h->res_last = clk::now();
    return WBC_OK;
}
}  // namespace
extern "C" {

int32_t wbc_cycle(wbc_engine* h, const double* base_pose, const double* nu, const double* qj, const double* ref,
                  const uint8_t* contacts, const uint8_t* switching, uint32_t flags, double* tau, double* grf, double* x,
                  int32_t* status, int32_t* iters) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    if (h->n_modes) return fail(WBC_ERR_STATE, "wbc_cycle: mode hypotheses are set");
    if (!base_pose || !nu || !qj || !ref || !contacts || !switching) return fail(WBC_ERR_ARG, "wbc_cycle: null input");
    WBC_HIP(hipSetDevice(h->device));
    const size_t B = (size_t)h->batch;
    const size_t inb = in_block_bytes(B), outb = out_block_bytes(B);
    if (!h->h_in) {
        WBC_HIP(hipHostMalloc(&h->h_in, (inb + 7) / 8 * 8, hipHostMallocMapped));  // (whole words: the resident copy)
        WBC_HIP(hipHostMalloc(&h->h_out, outb, hipHostMallocMapped));
#ifndef WBC_CYCLE_COPY  // (A/B builds only: the copy cycle at every batch size)
        // Small batches (the B = 1 drop-in) run zero-copy: the step reads the pinned input block and
        // writes the pinned output block through their device addresses (a few hundred bytes over
        // PCIe inside the kernel instead of an H2D and a D2H copy, each a separate queued operation).
        if (B <= kZeroCopyMaxBatch) {
            void *mi = nullptr, *mo = nullptr, *mq = nullptr;
            if (hipHostGetDevicePointer(&mi, h->h_in, 0) == hipSuccess &&
                hipHostGetDevicePointer(&mo, h->h_out, 0) == hipSuccess &&
                hipHostGetDevicePointer(&mq, h->h_qmap, 0) == hipSuccess) {
                h->m_in = mi;
                h->m_out = mo;
                h->m_qmap = static_cast<const int32_t*>(mq);
                h->m_contacts = reinterpret_cast<const uint8_t*>(static_cast<const double*>(mi) +
                                                                 B * (WBC_POSE_LEN + WBC_NU_LEN + WBC_NUM_JOINTS + WBC_REF_LEN));
            }
            (void)hipGetLastError();
        }
#endif
    }
    // pack the host inputs in the device block's layout (pinned), one H2D copy
    double* hp = static_cast<double*>(h->h_in);
    std::memcpy(hp, base_pose, B * WBC_POSE_LEN * sizeof(double));
    hp += B * WBC_POSE_LEN;
    std::memcpy(hp, nu, B * WBC_NU_LEN * sizeof(double));
    hp += B * WBC_NU_LEN;
    std::memcpy(hp, qj, B * WBC_NUM_JOINTS * sizeof(double));
    hp += B * WBC_NUM_JOINTS;
    std::memcpy(hp, ref, B * WBC_REF_LEN * sizeof(double));
    hp += B * WBC_REF_LEN;
    std::memcpy(reinterpret_cast<uint8_t*>(hp), contacts, B);
    std::memcpy(reinterpret_cast<uint8_t*>(hp) + B, switching, B);
    h->n_stance_own = count_stance(contacts, B);  // d_contacts holds these masks from here on
    h->qmap_waves = wbc::qmap_build(contacts, h->batch, h->h_qmap);  // uploaded by enqueue_cycle
    h->qmap_host = true;
    if (!x) flags |= WBC_NO_X;
    if ((flags & WBC_RESIDENT) && h->m_in && B <= (size_t)wbc::QMAP_SEG && !(flags & (WBC_SPLIT | WBC_FUSED | WBC_DEBUG))) {
        const int32_t rc = resident_cycle(h, flags & ~WBC_RESIDENT);
        if (rc != WBC_OK) return rc;
    } else {
        if (h->res_on) WBC_HIP(resident_stop(h));
        const int32_t rc = enqueue_cycle(h, flags & ~WBC_RESIDENT);
        if (rc != WBC_OK) return rc;
        WBC_HIP(hipStreamSynchronize(h->stream));
    }
    const size_t xb = B * WBC_NV * sizeof(double);
    const double* o = static_cast<const double*>(h->h_out);
    if (tau) std::memcpy(tau, o, B * WBC_NUM_JOINTS * sizeof(double));
    if (grf) std::memcpy(grf, o + B * WBC_NUM_JOINTS, B * WBC_NUM_JOINTS * sizeof(double));
    const int32_t* oi = reinterpret_cast<const int32_t*>(o + 2 * B * WBC_NUM_JOINTS);
    if (status) std::memcpy(status, oi, B * sizeof(int32_t));
    if (iters) std::memcpy(iters, oi + B, B * sizeof(int32_t));
    if (x) std::memcpy(x, reinterpret_cast<const double*>(oi + 2 * B), xb);
    return WBC_OK;
}

int32_t wbc_synchronize(wbc_engine* h) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(hipSetDevice(h->device));
    WBC_HIP(hipStreamSynchronize(h->stream));
    return WBC_OK;
}

int32_t wbc_get_output(wbc_engine* h, double* tau, double* grf, double* x, int32_t* status, int32_t* iters) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    WBC_HIP(hipSetDevice(h->device));
    const size_t B = (size_t)h->batch;
    hipStream_t st = h->stream;
    if (tau) WBC_HIP(hipMemcpyAsync(tau, h->out_tau, B * 12 * sizeof(double), hipMemcpyDeviceToHost, st));
    if (grf) WBC_HIP(hipMemcpyAsync(grf, h->out_grf, B * 12 * sizeof(double), hipMemcpyDeviceToHost, st));
    if (x) WBC_HIP(hipMemcpyAsync(x, h->out_x, B * WBC_NV * sizeof(double), hipMemcpyDeviceToHost, st));
    if (status) WBC_HIP(hipMemcpyAsync(status, h->out_status, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (iters) WBC_HIP(hipMemcpyAsync(iters, h->out_iters, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    WBC_HIP(hipStreamSynchronize(st));
    return WBC_OK;
}

int32_t wbc_device_outputs(wbc_engine* h, double** d_tau, double** d_grf, double** d_x, int32_t** d_status,
                           int32_t** d_iters) {
    if (!h) return fail(WBC_ERR_ARG, "null handle");
    WBC_HIP(sync_own(h));
    if (d_tau) *d_tau = h->out_tau;
    if (d_grf) *d_grf = h->out_grf;
    if (d_x) *d_x = h->out_x;
    if (d_status) *d_status = h->out_status;
    if (d_iters) *d_iters = h->out_iters;
    return WBC_OK;
}

int32_t wbc_get_debug(wbc_engine* h, double* out) {
    if (!h || !out) return fail(WBC_ERR_ARG, "null argument");
    WBC_HIP(hipSetDevice(h->device));
    WBC_HIP(hipMemcpyAsync(out, h->d_dbg, (size_t)h->batch * WBC_DBG_LEN * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    WBC_HIP(hipStreamSynchronize(h->stream));
    return WBC_OK;
}

int32_t wbc_modes_per_wave(wbc_engine* h, int32_t* m) {
    if (!h || !m) return fail(WBC_ERR_ARG, "null handle or output");
    *m = h->n_modes ? h->mode_loop : 0;
    return WBC_OK;
}

int32_t wbc_last_kernel_ms(wbc_engine* h, double* ms) {
    if (!h || !ms) return fail(WBC_ERR_ARG, "null argument");
    if (!h->timed) return fail(WBC_ERR_STATE, "no wbc_step ran with WBC_TIMED");
    float f = 0.f;
    WBC_HIP(hipEventSynchronize(h->ev1));
    WBC_HIP(hipEventElapsedTime(&f, h->ev0, h->ev1));
    *ms = (double)f;
    return WBC_OK;
}

const char* wbc_last_error(void) { return g_err.c_str(); }

// shared with the planner's C-ABI (wbc_planner.hip): one error string per thread for the library
void wbc_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }

}  // extern "C"
