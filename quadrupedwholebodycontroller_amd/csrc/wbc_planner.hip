// wbc_planner.hip — batched motion planner for gfx950: one robot per thread, one kernel launch
// per planner tick.  Restates src/motion_planner.cpp:1-383 (see include/wbc_planner.h for the
// interface mapping).  The reference's nested plannerLoop (cpp:171-376) becomes a per-robot state
// machine with one transition per `rate.sleep()`:
//
//   mode OUTER  evaluate the command (cpp:186): zero -> publish with all feet in contact
//               (cpp:366-369); non-zero -> start a 4-step cycle (cpp:188-210) and run its first
//               inner iteration in the same tick
//   mode INNER  one iteration of `while (step_phase < 4)` (cpp:212-356): publish the swing-foot
//               Bezier point of the phase's leg and the CoM segment (quintic timing), or, when the
//               phase time is up, advance the phase without publishing (cpp:351-355); after the 4th
//               phase the cycle bookkeeping (cpp:359-365) runs and the next tick is mode CYCLE_END
//   mode CYCLE_END  the outer loop's own sleep after a cycle (cpp:372-373): publishes nothing
//
// Arithmetic follows the reference expression by expression in fp64 (the phase clock is the same
// running sum of dt, so phase changes land on the same ticks).
#include <hip/hip_runtime.h>

#include <cmath>
#include <new>
#include <string>

#include "wbc_planner.h"

extern "C" void wbc_internal_set_error(const char* msg);

namespace wbcp {

enum Mode { OUTER = 0, INNER = 1, CYCLE_END = 2 };

// per-robot planner state (the MotionPlanner members, hpp:21-50, plus plannerLoop's locals)
struct State {
    double cmd[3];          // velocity_command_ x, y (z stays 0, cpp:123-124); [2] = yaw_rate_command_
    double yaw;
    double step_time, cycle_time;
    double vcr[3];          // velocity_command_rotated of the running cycle (cpp:191)
    double pi_body[3], pf_body[3];
    double pi_foot[4][3], pf_foot[4][3];  // planner order LH, RH, LF, RF
    double msg[54];         // ref_msg_ (WbcReferenceMsg field order)
    int32_t mode, step_phase, cycle_counter, contacts, last_published;
    int32_t pad;
};
static_assert(sizeof(State) % 8 == 0, "State layout");

struct Quintic {
    double a0, a1, a2, a3, a4, a5;
};
__device__ __forceinline__ Quintic quintic(double T, double vi, double vf) {  // cpp:68-97
    const double T2 = T * T, T3 = T2 * T, T4 = T3 * T, T5 = T4 * T;
    Quintic p;
    p.a0 = 0.0;
    p.a1 = vi;
    p.a2 = 0.0;
    p.a3 = (10.0 - 4.0 * vf * T - 6.0 * vi * T) / T3;
    p.a4 = (-15.0 + 7.0 * vf * T + 8.0 * vi * T) / T4;
    p.a5 = (6.0 - 3.0 * vf * T - 3.0 * vi * T) / T5;
    return p;
}
__device__ __forceinline__ void q_eval(const Quintic& a, double t, double& s, double& sd, double& sdd) {  // cpp:52-62
    s = a.a0 + a.a1 * t + a.a2 * t * t + a.a3 * t * t * t + a.a4 * t * t * t * t + a.a5 * t * t * t * t * t;
    sd = a.a1 + 2.0 * a.a2 * t + 3.0 * a.a3 * t * t + 4.0 * a.a4 * t * t * t + 5.0 * a.a5 * t * t * t * t;
    sdd = 2.0 * a.a2 + 6.0 * a.a3 * t + 12.0 * a.a4 * t * t + 20.0 * a.a5 * t * t * t;
}

// cubic Bezier through pi, pi + h z, pf + h z, pf and its first two s-derivatives (cpp:4-49)
__device__ __forceinline__ void bezier3(double s, const double* pi, const double* pf, double h, double* p, double* d1,
                                        double* d2) {
    const double oms = 1.0 - s;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double p0 = pi[i], p3 = pf[i];
        const double p1 = pi[i] + (i == 2 ? h : 0.0), p2 = pf[i] + (i == 2 ? h : 0.0);
        double v = (1 - s) * (1 - s) * (1 - s) * p0;
        v += 3 * (1 - s) * (1 - s) * s * p1;
        v += 3 * (1 - s) * s * s * p2;
        v += s * s * s * p3;
        p[i] = v;
        d1[i] = 3.0 * (oms * oms * (p1 - p0) + 2.0 * oms * s * (p2 - p1) + s * s * (p3 - p2));
        d2[i] = 6.0 * (oms * (p2 - 2.0 * p1 + p0) + s * (p3 - 2.0 * p2 + p1));
    }
}

// message leg (LH, LF, RF, RH) swung in step phase 0..3 (LH, RH, LF, RF; cpp:232-300)
__device__ __forceinline__ int swing_leg(int phase) { return phase == 0 ? 0 : (phase == 1 ? 3 : (phase == 2 ? 1 : 2)); }
// footContacts bitmask (bit i = message leg i) of step phase 0..3
__device__ __forceinline__ int phase_contacts(int phase) { return 15 & ~(1 << swing_leg(phase)); }

__device__ void reset_state(State& st, const wbc_planner_params& p) {  // constructor, cpp:129-168
    for (int i = 0; i < 3; ++i) { st.cmd[i] = 0.0; st.vcr[i] = 0.0; }
    st.yaw = 0.0;
    st.step_time = 0.0;
    st.cycle_time = 0.0;
    for (int i = 0; i < 54; ++i) st.msg[i] = 0.0;
    st.msg[2] = p.body_height;
    st.pi_body[0] = 0.0; st.pi_body[1] = 0.0; st.pi_body[2] = p.body_height;
    for (int i = 0; i < 3; ++i) st.pf_body[i] = st.pi_body[i] + p.step_length * 0.0;  // command is 0 here
    const double LH[3] = {st.pi_body[0] - p.x_offset, st.pi_body[1] + p.y_offset, 0.0};
    const double dir[4][3] = {{0.0, 0.0, 0.0}, {0.0, -2 * p.y_offset, 0.0}, {2 * p.x_offset, 0.0, 0.0},
                              {2 * p.x_offset, -2 * p.y_offset, 0.0}};  // LH, RH, LF, RF
    for (int f = 0; f < 4; ++f)
        for (int i = 0; i < 3; ++i) {
            st.pi_foot[f][i] = LH[i] + dir[f][i];
            st.pf_foot[f][i] = st.pi_foot[f][i];
        }
    st.mode = OUTER;
    st.step_phase = 0;
    st.cycle_counter = 0;
    st.contacts = 15;
    st.last_published = 15;  // the controller's initial footContacts_ (cpp:67-70)
    st.pad = 0;
}

__global__ void planner_reset_kernel(State* states, const uint8_t* mask, wbc_planner_params p, int batch) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch || (mask && !mask[b])) return;
    reset_state(states[b], p);
}

__global__ void planner_tick_kernel(State* states, wbc_planner_params p, int batch, double* ref_out,
                                    uint8_t* contacts_out, uint8_t* switching_out, uint8_t* published_out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    State st = states[b];
    const double cycle_duration = 4 * p.step_duration;  // cpp:119
    bool published = false;

    if (st.mode == CYCLE_END) {
        st.mode = OUTER;  // the outer loop's sleep after a cycle: nothing published
    } else {
        if (st.mode == OUTER) {
            const bool moving = (st.cmd[0] != 0.0 || st.cmd[1] != 0.0) || st.cmd[2] != 0;
            if (!moving) {  // stand still: all feet in contact, rest of the message unchanged
                st.contacts = 15;
                published = true;
            } else {        // start of a 4-step cycle (cpp:188-210)
                const double cy = cos(st.yaw), sy = sin(st.yaw);
                // rot_matrix * velocity_command_ (z component of the command is 0)
                st.vcr[0] = cy * st.cmd[0] + -sy * st.cmd[1] + 0 * 0.0;
                st.vcr[1] = sy * st.cmd[0] + cy * st.cmd[1] + 0 * 0.0;
                st.vcr[2] = 0 * st.cmd[0] + 0 * st.cmd[1] + 1 * 0.0;
                const double dyaw = st.cmd[2] * cycle_duration;
                const double cd = cos(dyaw), sd = sin(dyaw);
                for (int f = 0; f < 4; ++f) {
                    const double vx = st.pi_foot[f][0] - st.pi_body[0], vy = st.pi_foot[f][1] - st.pi_body[1];
                    const double dn[3] = {(cd * vx + -sd * vy + 0 * 0.0) - vx, (sd * vx + cd * vy + 0 * 0.0) - vy,
                                          (0 * vx + 0 * vy + 1 * 0.0) - 0.0};
                    for (int i = 0; i < 3; ++i) st.pf_foot[f][i] += st.vcr[i] * p.step_length + dn[i];
                }
                st.mode = INNER;
            }
        }
        if (st.mode == INNER) {
            if (st.step_time < p.step_duration) {  // cpp:213-349
                const Quintic pf_ = quintic(p.step_duration, 0.0, 0.0);
                double s, sdt, sddt;
                q_eval(pf_, st.step_time, s, sdt, sddt);
                double pt[3], d1[3], d2[3];
                const int ph = st.step_phase;
                bezier3(s, st.pi_foot[ph], st.pf_foot[ph], p.height_control_point, pt, d1, d2);
                const int leg = swing_leg(ph);
                for (int i = 0; i < 3; ++i) {
                    st.msg[18 + 3 * leg + i] = pt[i];
                    st.msg[30 + 3 * leg + i] = d1[i] * sdt;
                    st.msg[42 + 3 * leg + i] = d2[i] * sdt * sdt + d1[i] * sddt;
                }
                st.contacts = phase_contacts(ph);
                const Quintic pb = (st.cycle_counter == 0) ? quintic(cycle_duration, 0.0, p.body_final_velocity)
                                                           : quintic(cycle_duration, p.body_final_velocity,
                                                                     p.body_final_velocity);
                double sb, sbd, sbdd;
                q_eval(pb, st.cycle_time, sb, sbd, sbdd);
                for (int i = 0; i < 3; ++i) {
                    const double dp = st.pf_body[i] - st.pi_body[i];
                    st.msg[i] = st.pi_body[i] + sb * dp;
                    st.msg[6 + i] = dp * sbd;
                    st.msg[12 + i] = dp * sbdd;
                }
                st.msg[3] = 0.0; st.msg[4] = 0.0; st.msg[5] = st.yaw;
                st.msg[9] = 0.0; st.msg[10] = 0.0; st.msg[11] = st.cmd[2];
                st.msg[15] = 0.0; st.msg[16] = 0.0; st.msg[17] = 0.0;
                published = true;
                st.yaw += st.cmd[2] * p.dt;
                st.step_time += p.dt;
                st.cycle_time += p.dt;
            } else {  // phase time is up: next phase, nothing published (cpp:351-355)
                st.step_phase += 1;
                st.step_time = 0.0;
                if (st.step_phase == 4) {  // end of the 4-step cycle (cpp:358-365)
                    st.cycle_counter += 1;
                    st.step_phase = 0;
                    st.cycle_time = 0.0;
                    for (int i = 0; i < 3; ++i) {
                        st.pi_body[i] = st.pf_body[i];
                        st.pf_body[i] += st.vcr[i] * p.step_length;
                    }
                    for (int f = 0; f < 4; ++f)
                        for (int i = 0; i < 3; ++i) st.pi_foot[f][i] = st.pf_foot[f][i];
                    st.mode = CYCLE_END;
                }
            }
        }
    }
    if (published) {
        for (int i = 0; i < 54; ++i) ref_out[(size_t)b * 54 + i] = st.msg[i];
        contacts_out[b] = (uint8_t)st.contacts;
        switching_out[b] = (uint8_t)(st.contacts != st.last_published);
        st.last_published = st.contacts;
    }
    published_out[b] = published ? 1 : 0;
    states[b] = st;
}

__global__ void planner_command_kernel(State* states, const double* cmd, int batch) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    for (int i = 0; i < 3; ++i) states[b].cmd[i] = cmd[(size_t)b * 3 + i];
}

}  // namespace wbcp

struct wbc_planner {
    int32_t batch = 0, device = 0;
    wbc_planner_params params{};
    hipStream_t own_stream = nullptr, stream = nullptr;
    wbcp::State* d_state = nullptr;
    double* d_cmd = nullptr;
    double* d_ref = nullptr;
    uint8_t* d_contacts = nullptr;
    uint8_t* d_switching = nullptr;
    uint8_t* d_published = nullptr;
    uint8_t* d_mask = nullptr;
};

namespace {
constexpr int kThreads = 256;
int32_t pfail(int32_t code, const std::string& m) {
    wbc_internal_set_error(m.c_str());
    return code;
}
#define P_HIP(call)                                                                                  \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess) return pfail(-2, std::string(#call ": ") + hipGetErrorString(e_));     \
    } while (0)
int blocks(int b) { return (b + kThreads - 1) / kThreads; }
}  // namespace

extern "C" {

int32_t wbc_planner_default_params(wbc_planner_params* o) {
    if (!o) return pfail(-1, "null argument");
    o->step_length = 0.1;          // params_planner.yaml:1
    o->height_control_point = 0.1; // :2
    o->x_offset = 0.50;            // :3
    o->y_offset = 0.33;            // :4
    o->step_duration = 0.2;        // :5
    o->body_height = 0.50;         // :6
    o->body_initial_velocity = 0.0;
    o->body_final_velocity = 0.40; // :7
    o->dt = 0.01;                  // :8
    return 0;
}

int32_t wbc_planner_destroy(wbc_planner* h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    (void)hipFree(h->d_state);
    (void)hipFree(h->d_cmd);
    (void)hipFree(h->d_ref);
    (void)hipFree(h->d_contacts);
    (void)hipFree(h->d_switching);
    (void)hipFree(h->d_published);
    (void)hipFree(h->d_mask);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return 0;
}

int32_t wbc_planner_create(const wbc_planner_params* params, int32_t batch, int32_t device, wbc_planner** out) {
    if (!out || batch <= 0) return pfail(-1, "wbc_planner_create: bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return pfail(-4, "no HIP device");
    if (device < 0 || device >= ndev) return pfail(-1, "wbc_planner_create: bad device index");
    P_HIP(hipSetDevice(device));
    wbc_planner* h = new (std::nothrow) wbc_planner();
    if (!h) return pfail(-1, "out of host memory");
    h->batch = batch;
    h->device = device;
    if (params) h->params = *params;
    else wbc_planner_default_params(&h->params);
    const size_t B = (size_t)batch;
    hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_state), B * sizeof(wbcp::State));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_cmd), B * 3 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_ref), B * 54 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_contacts), B);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_switching), B);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_published), B);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->d_mask), B);
    if (e != hipSuccess) {
        wbc_planner_destroy(h);
        return pfail(-2, std::string("wbc_planner_create: ") + hipGetErrorString(e));
    }
    h->stream = h->own_stream;
    // the initial message is what the controller would hold before the first publication
    P_HIP(hipMemsetAsync(h->d_ref, 0, B * 54 * sizeof(double), h->stream));
    P_HIP(hipMemsetAsync(h->d_contacts, 15, B, h->stream));
    P_HIP(hipMemsetAsync(h->d_switching, 0, B, h->stream));
    P_HIP(hipMemsetAsync(h->d_published, 0, B, h->stream));
    hipLaunchKernelGGL(wbcp::planner_reset_kernel, dim3(blocks(batch)), dim3(kThreads), 0, h->stream, h->d_state,
                       (const uint8_t*)nullptr, h->params, batch);
    P_HIP(hipGetLastError());
    P_HIP(hipStreamSynchronize(h->stream));
    *out = h;
    return 0;
}

int32_t wbc_planner_set_stream(wbc_planner* h, void* s) {
    if (!h) return pfail(-1, "null handle");
    h->stream = s ? reinterpret_cast<hipStream_t>(s) : h->own_stream;
    return 0;
}

int32_t wbc_planner_set_command(wbc_planner* h, const double* cmd) {
    if (!h || !cmd) return pfail(-1, "null argument");
    P_HIP(hipSetDevice(h->device));
    P_HIP(hipMemcpyAsync(h->d_cmd, cmd, (size_t)h->batch * 3 * sizeof(double), hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(wbcp::planner_command_kernel, dim3(blocks(h->batch)), dim3(kThreads), 0, h->stream, h->d_state,
                       (const double*)h->d_cmd, h->batch);
    P_HIP(hipGetLastError());
    P_HIP(hipStreamSynchronize(h->stream));  // the host array may be reused by the caller
    return 0;
}

int32_t wbc_planner_reset(wbc_planner* h, const uint8_t* mask) {
    if (!h) return pfail(-1, "null handle");
    P_HIP(hipSetDevice(h->device));
    const uint8_t* dm = nullptr;
    if (mask) {
        P_HIP(hipMemcpyAsync(h->d_mask, mask, (size_t)h->batch, hipMemcpyHostToDevice, h->stream));
        dm = h->d_mask;
    }
    hipLaunchKernelGGL(wbcp::planner_reset_kernel, dim3(blocks(h->batch)), dim3(kThreads), 0, h->stream, h->d_state,
                       dm, h->params, h->batch);
    P_HIP(hipGetLastError());
    P_HIP(hipStreamSynchronize(h->stream));
    return 0;
}

int32_t wbc_planner_tick(wbc_planner* h) {
    if (!h) return pfail(-1, "null handle");
    P_HIP(hipSetDevice(h->device));
    hipLaunchKernelGGL(wbcp::planner_tick_kernel, dim3(blocks(h->batch)), dim3(kThreads), 0, h->stream, h->d_state,
                       h->params, h->batch, h->d_ref, h->d_contacts, h->d_switching, h->d_published);
    P_HIP(hipGetLastError());
    return 0;
}

int32_t wbc_planner_device_outputs(wbc_planner* h, double** ref, uint8_t** contacts, uint8_t** switching,
                                   uint8_t** published) {
    if (!h) return pfail(-1, "null handle");
    if (ref) *ref = h->d_ref;
    if (contacts) *contacts = h->d_contacts;
    if (switching) *switching = h->d_switching;
    if (published) *published = h->d_published;
    return 0;
}

int32_t wbc_planner_get_output(wbc_planner* h, double* ref, uint8_t* contacts, uint8_t* switching, uint8_t* published) {
    if (!h) return pfail(-1, "null handle");
    P_HIP(hipSetDevice(h->device));
    const size_t B = (size_t)h->batch;
    if (ref) P_HIP(hipMemcpyAsync(ref, h->d_ref, B * 54 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (contacts) P_HIP(hipMemcpyAsync(contacts, h->d_contacts, B, hipMemcpyDeviceToHost, h->stream));
    if (switching) P_HIP(hipMemcpyAsync(switching, h->d_switching, B, hipMemcpyDeviceToHost, h->stream));
    if (published) P_HIP(hipMemcpyAsync(published, h->d_published, B, hipMemcpyDeviceToHost, h->stream));
    P_HIP(hipStreamSynchronize(h->stream));
    return 0;
}

}  // extern "C"
