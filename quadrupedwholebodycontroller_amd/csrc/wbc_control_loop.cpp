// wbc_control_loop — ROS-free stand-in for whole_body_controller_node (src/whole_body_controller_node.cpp:3-9):
// drives the WholeBodyController shim (include/wbc_controller.hpp) through its callbacks and
// controlLoop(), one robot, on the GPU.
//
//   wbc_control_loop stance [cycles] [rate_hz]
//       BASELINE configs[0]: stance CoM-hold from the reference start-up pose (base 0.585 m, q0,
//       all feet in contact, reference pose from params_controller.yaml), `cycles` (default 1000)
//       control cycles; prints one JSON line with per-cycle latency and the last torques.
//   wbc_control_loop run [cycles]
//       the node's own entry, `WholeBodyController wbc; wbc.run();` (whole_body_controller_node.cpp:6-7):
//       the control thread runs back to back while this thread spins, publishing the stance
//       messages through the callbacks (ros::spin's role); a loop hook requests shutdown after
//       `cycles` (default 200).  Prints one JSON line (cycles, QP status, torques, messages sent).
//   wbc_control_loop replay <inputs.bin> <outputs.bin>
//       feeds recorded per-cycle messages (tests/test_gpu_controller.py writes them from the golden
//       trajectories) and writes status, iterations, tau and x per cycle.
//       inputs.bin : int32 T, then T x (pose 7, nu 18, qj 12, ref 54, contacts, switching) doubles
//       outputs.bin: T x (status, iters, tau 12, x 42) doubles
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "wbc_controller.hpp"

using namespace wbc_mi355x;

namespace {

constexpr int kRec = 7 + 18 + 12 + 54 + 2;
constexpr int kOut = 2 + 12 + 42;

// messages as the simulator / planner would publish them (cpp:150-254)
ModelStates make_model_states(const double* pose, const double* nu) {
    ModelStates m;
    m.name = {"ground_plane", WholeBodyController::modelName};
    m.pose.resize(2);
    m.twist.resize(2);
    Pose& p = m.pose[1];
    p.position = {pose[0], pose[1], pose[2]};
    p.orientation = {pose[3], pose[4], pose[5], pose[6]};
    m.twist[1].linear = {nu[0], nu[1], nu[2]};
    m.twist[1].angular = {nu[3], nu[4], nu[5]};
    return m;
}
JointState make_joint_state(const double* qj, const double* qd) {
    // alphabetical order (as robot_state_publisher emits), not the model order: exercises the
    // name mapping of jointStateCallback (cpp:234-246)
    JointState j;
    std::vector<int> order(numberOfJoints);
    for (int i = 0; i < numberOfJoints; ++i) order[i] = i;
    const auto& names = modelJointNames();
    std::sort(order.begin(), order.end(), [&](int a, int b) { return names[a] < names[b]; });
    for (int k : order) {
        j.name.push_back(names[k]);
        j.position.push_back(qj[k]);
        j.velocity.push_back(qd[k]);
        j.effort.push_back(0.0);
    }
    return j;
}
WbcReferenceMsg make_reference(const double* ref, int contacts) {
    WbcReferenceMsg r;
    r.desiredComPose.data.assign(ref, ref + 6);
    r.desiredComVelocity.data.assign(ref + 6, ref + 12);
    r.desiredComAcceleration.data.assign(ref + 12, ref + 18);
    r.desiredSwingLegsPosition.data.assign(ref + 18, ref + 30);
    r.desiredSwingLegsVelocity.data.assign(ref + 30, ref + 42);
    r.desiredSwingLegsAcceleration.data.assign(ref + 42, ref + 54);
    for (int l = 0; l < numberOfLegs; ++l) r.footContacts[l] = (contacts >> l) & 1;
    return r;
}

int run_stance(long cycles, double rate, uint32_t flags) {
    WholeBodyController wbc;
    wbc.setStepFlags(flags);
    double pose[7] = {0.0, 0.0, 0.585, 0.0, 0.0, 0.0, 1.0};
    double nu[18] = {0};
    const double q0[12] = {0.0, -0.4, 0.8, 0.0, 0.4, -0.8, 0.0, 0.4, -0.8, 0.0, -0.4, 0.8};
    wbc_params p;
    wbc_default_params(&p);
    double ref[54] = {0};
    for (int i = 0; i < 6; ++i) ref[i] = p.initial_reference_pose[i];
    const ModelStates ms = make_model_states(pose, nu);
    const JointState js = make_joint_state(q0, nu + 6);
    const WbcReferenceMsg rm = make_reference(ref, 15);
    wbc.floatingBaseStateCallback(ms);  // first message: locates the model only (cpp:189-204)
    std::vector<double> lat, work;
    lat.reserve(cycles);
    work.reserve(cycles);
    auto t_prev = std::chrono::steady_clock::now();
    long n = 0;
    auto feed = [&](long it) {
        const auto now = std::chrono::steady_clock::now();
        if (it > 0) lat.push_back(std::chrono::duration<double, std::micro>(now - t_prev).count());
        t_prev = now;
        wbc.floatingBaseStateCallback(ms);
        wbc.jointStateCallback(js);
        wbc.referenceCallback(rm);
    };
    if (rate > 0.0) {
        // a paced loop (ros::Rate): the same cycles as controlLoop, with each cycle's own time
        // (controlCycle alone, without the sleep) recorded as work_us; at rates below the resident
        // wave's restart limit (25 Hz) every cycle starts a new wave
        wbc.setInitialState();
        const auto period = std::chrono::duration_cast<std::chrono::steady_clock::duration>(
            std::chrono::duration<double>(1.0 / rate));
        auto next = std::chrono::steady_clock::now();
        for (; n < cycles; ++n) {
            feed(n);
            const auto t0 = std::chrono::steady_clock::now();
            wbc.controlCycle();
            work.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            if (wbc.qpReturnValue() != WBC_QP_OK) { ++n; break; }
            next += period;
            std::this_thread::sleep_until(next);
        }
    } else {
        n = wbc.controlLoop(cycles, rate, feed);
    }
    auto stats = [](std::vector<double> s, double& mean, double& p50, double& p99) {
        std::sort(s.begin(), s.end());
        auto pct = [&](double q) { return s.empty() ? 0.0 : s[std::min(s.size() - 1, (size_t)(q * s.size()))]; };
        mean = 0;
        for (double v : s) mean += v;
        mean = s.empty() ? 0 : mean / s.size();
        p50 = pct(0.5);
        p99 = pct(0.99);
    };
    double mean, p50, p99, wmean, w50, w99;
    stats(lat, mean, p50, p99);
    stats(work, wmean, w50, w99);
    const auto& tau = wbc.jointTorques();
    std::printf("{\"config\": \"stance_hold_b1\", \"cycles\": %ld, \"qp_status\": %d, \"qp_iters\": %d, "
                "\"cycle_us_mean\": %.3f, \"cycle_us_p50\": %.3f, \"cycle_us_p99\": %.3f, \"rate_hz\": %.1f, ",
                n, wbc.qpReturnValue(), wbc.qpIterations(), mean, p50, p99, rate);
    if (rate > 0.0) std::printf("\"work_us_mean\": %.3f, \"work_us_p50\": %.3f, \"work_us_p99\": %.3f, ", wmean, w50, w99);
    std::printf("\"tau\": [");
    for (int i = 0; i < numberOfJoints; ++i) std::printf("%s%.9g", i ? ", " : "", tau[i]);
    std::printf("]}\n");
    return wbc.qpReturnValue() == WBC_QP_OK ? 0 : 3;
}

int run_node(long cycles) {
    WholeBodyController wbc;  // the node's two statements (whole_body_controller_node.cpp:6-7) ...
    wbc.setRunRate(0.0);      // ... back to back instead of at 400 Hz
    double pose[7] = {0.0, 0.0, 0.585, 0.0, 0.0, 0.0, 1.0};
    double nu[18] = {0};
    const double q0[12] = {0.0, -0.4, 0.8, 0.0, 0.4, -0.8, 0.0, 0.4, -0.8, 0.0, -0.4, 0.8};
    wbc_params p;
    wbc_default_params(&p);
    double ref[54] = {0};
    for (int i = 0; i < 6; ++i) ref[i] = p.initial_reference_pose[i];
    const ModelStates ms = make_model_states(pose, nu);
    const JointState js = make_joint_state(q0, nu + 6);
    const WbcReferenceMsg rm = make_reference(ref, 15);
    wbc.floatingBaseStateCallback(ms);  // locates the model (cpp:189-204)
    std::atomic<long> sent{0};
    wbc.spinOnce = [&]() {  // the subscriber callbacks, concurrently with the control thread
        wbc.floatingBaseStateCallback(ms);
        wbc.jointStateCallback(js);
        wbc.referenceCallback(rm);
        sent.fetch_add(1);
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    };
    wbc.loopHook = [&](long it) {
        if (it + 1 >= cycles) wbc.requestShutdown();  // ros::shutdown: this cycle is the last
    };
    const long n = wbc.run();
    const auto tau = wbc.jointTorques();  // (a copy: the loop below publishes new torques)
    const int status = wbc.qpReturnValue();
    auto feed = [&](long) {
        wbc.floatingBaseStateCallback(ms);
        wbc.jointStateCallback(js);
        wbc.referenceCallback(rm);
    };
    // after run() ended by requestShutdown(), ok() stays false (ros::ok(), cpp:648): a direct
    // controlLoop() runs no cycle until resetShutdown() clears the request
    const long halted = wbc.controlLoop(25, 0.0, feed);
    wbc.resetShutdown();
    const long again = wbc.controlLoop(25, 0.0, feed);
    // a shutdown requested before run() is not dropped by run() either: it runs no cycle
    wbc.requestShutdown();
    wbc.loopHook = nullptr;
    const long pre = wbc.run();
    wbc.resetShutdown();
    std::printf("{\"config\": \"node_run\", \"cycles\": %ld, \"control_loop_after_shutdown\": %ld, "
                "\"control_loop_after_run\": %ld, \"run_after_request\": %ld, \"qp_status\": %d, "
                "\"messages\": %ld, \"tau\": [", n, halted, again, pre, status, sent.load());
    for (int i = 0; i < numberOfJoints; ++i) std::printf("%s%.9g", i ? ", " : "", tau[i]);
    std::printf("]}\n");
    return status == WBC_QP_OK && wbc.qpReturnValue() == WBC_QP_OK ? 0 : 3;
}

int run_replay(const char* in_path, const char* out_path) {
    FILE* f = std::fopen(in_path, "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + in_path);
    int32_t T = 0;
    if (std::fread(&T, sizeof(T), 1, f) != 1 || T <= 0) throw std::runtime_error("bad header");
    std::vector<double> in((size_t)T * kRec);
    if (std::fread(in.data(), sizeof(double), in.size(), f) != in.size()) throw std::runtime_error("short input");
    std::fclose(f);
    std::vector<double> out((size_t)T * kOut, 0.0);
    WholeBodyController wbc;
    {
        const double* r = in.data();
        wbc.floatingBaseStateCallback(make_model_states(r, r + 7));  // locate the model
    }
    const long n = wbc.controlLoop(T, 0.0, [&](long t) {
        const double* r = in.data() + (size_t)t * kRec;
        wbc.floatingBaseStateCallback(make_model_states(r, r + 7));
        wbc.jointStateCallback(make_joint_state(r + 25, r + 13));
        wbc.referenceCallback(make_reference(r + 37, (int)r[91]));
        if ((r[92] != 0.0) != wbc.isSwitchingFootState())
            throw std::runtime_error("isSwitchingFootState_ latch differs from the recorded input");
    });
    // controlLoop stops at a failed QP; record what ran
    (void)n;
    FILE* g = std::fopen(out_path, "wb");
    if (!g) throw std::runtime_error(std::string("cannot open ") + out_path);
    // re-run cycle by cycle to capture every output (the loop above validates the latch and the stop rule)
    WholeBodyController w2;
    w2.floatingBaseStateCallback(make_model_states(in.data(), in.data() + 7));
    for (int t = 0; t < T; ++t) {
        const double* r = in.data() + (size_t)t * kRec;
        w2.floatingBaseStateCallback(make_model_states(r, r + 7));
        w2.jointStateCallback(make_joint_state(r + 25, r + 13));
        w2.referenceCallback(make_reference(r + 37, (int)r[91]));
        w2.updateState();
        w2.solveQP();
        w2.computeJointTorques();
        double* o = out.data() + (size_t)t * kOut;
        o[0] = w2.qpReturnValue();
        o[1] = w2.qpIterations();
        for (int i = 0; i < 12; ++i) o[2 + i] = w2.jointTorques()[i];
        for (int i = 0; i < 42; ++i) o[14 + i] = w2.qpSolution()[i];
    }
    std::fwrite(out.data(), sizeof(double), out.size(), g);
    std::fclose(g);
    std::printf("{\"replayed\": %d, \"control_loop_cycles\": %ld}\n", T, n);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        const std::string mode = argc > 1 ? argv[1] : "stance";
        if (mode == "stance")
            return run_stance(argc > 2 ? std::atol(argv[2]) : 1000, argc > 3 ? std::atof(argv[3]) : 0.0,
                              (argc > 4 && std::string(argv[4]) == "fused") ? WBC_FUSED
                              : (argc > 4 && std::string(argv[4]) == "split") ? WBC_SPLIT
                              : (argc > 4 && std::string(argv[4]) == "launch") ? 0u  // a kernel launch per cycle
                              : WBC_RESIDENT);  // "default" or nothing: the shim's default, the resident step
        if (mode == "replay" && argc > 3) return run_replay(argv[2], argv[3]);
        if (mode == "run") return run_node(argc > 2 ? std::atol(argv[2]) : 200);
        std::fprintf(stderr, "usage: %s stance [cycles] [rate_hz] [fused|split|launch|default] | run [cycles] | replay <in.bin> <out.bin>\n",
                     argv[0]);
        return 2;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "wbc_control_loop: %s\n", e.what());
        return 1;
    }
}
