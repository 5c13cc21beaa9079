// wbc_controller.cpp — the reference's WholeBodyController surface over the C-ABI engine (B = 1).
// See include/wbc_controller.hpp for the method-by-method mapping to the reference.
#include "wbc_controller.hpp"

#include <chrono>
#include <climits>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <thread>

namespace wbc_mi355x {

namespace {
void check(int32_t rc, const char* what) {
    if (rc != WBC_OK) throw std::runtime_error(std::string(what) + ": " + wbc_last_error());
}
// q0 of setInitialState (cpp:81), model order
constexpr double kInitialJointPos[numberOfJoints] = {0.0, -0.4, 0.8, 0.0, 0.4, -0.8, 0.0, 0.4, -0.8, 0.0, -0.4, 0.8};
}  // namespace

const std::array<std::string, numberOfJoints>& modelJointNames() {
    static const std::array<std::string, numberOfJoints> names = {
        "LH_HAA", "LH_HFE", "LH_KFE", "LF_HAA", "LF_HFE", "LF_KFE",
        "RF_HAA", "RF_HFE", "RF_KFE", "RH_HAA", "RH_HFE", "RH_KFE"};
    return names;
}

WholeBodyController::WholeBodyController(const wbc_params* params, int device) {
    if (params) params_ = *params;
    else check(wbc_default_params(&params_), "wbc_default_params");  // loadParameters (cpp:122-148)
    wbc_model model;
    check(wbc_anymal_model(&model), "wbc_anymal_model");  // ModelLoader + KinDynComputations (cpp:26-40)
    check(wbc_create(&model, &params_, 1, device, &engine_), "wbc_create");
    setInitialState();
}

WholeBodyController::~WholeBodyController() {
    if (engine_) wbc_destroy(engine_);
}

void WholeBodyController::setInitialState() {
    // cpp:65-120: all feet in contact, identity attitude at z = 0.60, q0, zero velocities,
    // desiredPose_ = initialReferencePose, other references zero, history reset
    std::lock_guard<std::mutex> lk(mu_);
    for (int i = 0; i < numberOfLegs; ++i) footContacts_[i] = 1;
    std::memset(basePose_, 0, sizeof(basePose_));
    basePose_[2] = 0.60;
    basePose_[6] = 1.0;
    std::memset(nu_, 0, sizeof(nu_));
    std::memcpy(jointPos_, kInitialJointPos, sizeof(jointPos_));
    std::memset(ref_, 0, sizeof(ref_));
    for (int i = 0; i < 6; ++i) ref_[i] = params_.initial_reference_pose[i];
    isSwitchingFootState_ = false;  // hpp:151
    firstControllerIteration_ = true;
    check(wbc_reset(engine_, nullptr), "wbc_reset");  // T_old = I, J_old = 0, e_int = 0, Tdot_inv = 0
}

void WholeBodyController::floatingBaseStateCallback(const ModelStates& msg) {
    // cpp:187-230: the first message only locates the model (and is otherwise ignored)
    std::lock_guard<std::mutex> lk(mu_);
    if (firstFloatingBaseStateCallback_) {
        modelIndex_ = 0;
        while (modelIndex_ < (int)msg.name.size() && msg.name[modelIndex_] != modelName) ++modelIndex_;
        firstFloatingBaseStateCallback_ = false;
        return;
    }
    if (modelIndex_ >= (int)msg.pose.size() || modelIndex_ >= (int)msg.twist.size())
        throw std::out_of_range("floatingBaseStateCallback: model not present in ModelStates");
    const Pose& p = msg.pose[modelIndex_];
    const Twist& t = msg.twist[modelIndex_];
    basePose_[0] = p.position.x; basePose_[1] = p.position.y; basePose_[2] = p.position.z;
    basePose_[3] = p.orientation.x; basePose_[4] = p.orientation.y; basePose_[5] = p.orientation.z;
    basePose_[6] = p.orientation.w;
    nu_[0] = t.linear.x; nu_[1] = t.linear.y; nu_[2] = t.linear.z;      // baseVel_ = [lin; ang]
    nu_[3] = t.angular.x; nu_[4] = t.angular.y; nu_[5] = t.angular.z;
}

void WholeBodyController::jointStateCallback(const JointState& msg) {
    // cpp:232-254: map message order to model order by name on the first message
    std::lock_guard<std::mutex> lk(mu_);
    if (firstJointStateCallback_) {
        const auto& names = modelJointNames();
        for (int i = 0; i < numberOfJoints; ++i) {
            int k = 0;
            while (k < (int)msg.name.size() && msg.name[k] != names[i]) ++k;
            if (k == (int)msg.name.size()) throw std::invalid_argument("jointStateCallback: missing joint " + names[i]);
            jointIndex_[i] = k;
        }
        firstJointStateCallback_ = false;
    }
    for (int i = 0; i < numberOfJoints; ++i) {
        jointPos_[i] = msg.position.at(jointIndex_[i]);
        nu_[6 + i] = msg.velocity.at(jointIndex_[i]);
    }
}

void WholeBodyController::referenceCallback(const WbcReferenceMsg& m) {
    // cpp:150-185; isSwitchingFootState_ latches per message
    const Float64MultiArray* f[6] = {&m.desiredComPose, &m.desiredComVelocity, &m.desiredComAcceleration,
                                     &m.desiredSwingLegsPosition, &m.desiredSwingLegsVelocity,
                                     &m.desiredSwingLegsAcceleration};
    const int n[6] = {6, 6, 6, 12, 12, 12};
    for (int b = 0; b < 6; ++b)
        if ((int)f[b]->data.size() < n[b]) throw std::invalid_argument("referenceCallback: short field");
    std::lock_guard<std::mutex> lk(mu_);
    int off = 0;
    for (int b = 0; b < 6; ++b) {
        for (int i = 0; i < n[b]; ++i) ref_[off + i] = f[b]->data[i];
        off += n[b];
    }
    isSwitchingFootState_ = false;
    for (int i = 0; i < numberOfLegs; ++i) {
        const int c = m.footContacts[i] ? 1 : 0;
        if (footContacts_[i] != c) isSwitchingFootState_ = true;
        footContacts_[i] = c;
    }
}

WholeBodyController::Inputs WholeBodyController::snapshot() {
    std::lock_guard<std::mutex> lk(mu_);
    Inputs in;
    std::memcpy(in.basePose, basePose_, sizeof(basePose_));
    std::memcpy(in.nu, nu_, sizeof(nu_));
    std::memcpy(in.jointPos, jointPos_, sizeof(jointPos_));
    std::memcpy(in.ref, ref_, sizeof(ref_));
    in.contacts = 0;
    for (int i = 0; i < numberOfLegs; ++i) in.contacts |= (uint8_t)(footContacts_[i] ? 1u << i : 0u);
    in.switching = isSwitchingFootState_ ? 1 : 0;
    return in;
}

void WholeBodyController::pushInputs() {
    const Inputs in = snapshot();
    check(wbc_set_state(engine_, in.basePose, in.nu, in.jointPos), "wbc_set_state");
    check(wbc_set_reference(engine_, in.ref, &in.contacts, &in.switching), "wbc_set_reference");
}

void WholeBodyController::updateState() {
    pushInputs();  // snapshot of the callback state for this cycle
    check(wbc_update(engine_, 0u), "wbc_update");
}

void WholeBodyController::solveQP() {
    // init on the first iteration, hotstart afterwards (cpp:523-535): the engine's dual active-set
    // solve reaches the same unique optimum either way (H is positive definite)
    check(wbc_solve(engine_, 0u), "wbc_solve");
    firstControllerIteration_ = false;
}

void WholeBodyController::computeJointTorques() {
    int32_t st = 0, it = 0;
    check(wbc_get_output(engine_, tau_.data(), grf_.data(), x_.data(), &st, &it), "wbc_get_output");
    qpStatus_ = st;
    qpIters_ = it;
    publish();
}

void WholeBodyController::controlCycle() {
    const Inputs in = snapshot();  // the callbacks may keep running while the engine steps
    int32_t st = 0, it = 0;
    check(wbc_cycle(engine_, in.basePose, in.nu, in.jointPos, in.ref, &in.contacts, &in.switching, stepFlags_, tau_.data(),
                    grf_.data(), x_.data(), &st, &it),
          "wbc_cycle");
    firstControllerIteration_ = false;
    qpStatus_ = st;
    qpIters_ = it;
    publish();
}

void WholeBodyController::publish() {
    // published before the caller checks the QP status, in the reference's order (cpp:652-659).
    // One difference: on a failed solve the reference publishes qpOASES' last iterate, the engine
    // publishes zeros (wbc.h, wbc_get_output); controlLoop then terminates either way.
    if (desiredGroundReactionForcesPublisher) {
        Float64MultiArray g;
        g.data.assign(grf_.begin(), grf_.end());
        desiredGroundReactionForcesPublisher(g);
    }
    if (jointTorquePublisher) {
        Float64MultiArray t;
        t.data.assign(tau_.begin(), tau_.end());
        jointTorquePublisher(t);
    }
}

void WholeBodyController::terminate() {
    // cpp:627-636: zero torque command
    if (jointTorquePublisher) {
        Float64MultiArray t;
        t.data.assign(numberOfJoints, 0.0);
        jointTorquePublisher(t);
    }
}

long WholeBodyController::controlLoop(long max_iterations, double rate_hz, const std::function<void(long)>& beforeCycle) {
    return loop(max_iterations, rate_hz, beforeCycle);  // shutdown_ as the caller left it (resetShutdown)
}

long WholeBodyController::loop(long max_iterations, double rate_hz, const std::function<void(long)>& beforeCycle) {
    setInitialState();  // resetRobotSimState (cpp:578-605) ends in setInitialState
    const auto period = rate_hz > 0 ? std::chrono::duration<double>(1.0 / rate_hz) : std::chrono::duration<double>(0);
    auto next = std::chrono::steady_clock::now();
    long iteration = 0;
    for (; iteration < max_iterations && ok(); ++iteration) {  // while (ros::ok()) (cpp:648)
        if (beforeCycle) beforeCycle(iteration);
        controlCycle();  // updateState(); solveQP(); computeJointTorques();
        if (qpStatus_ != WBC_QP_OK) {  // cpp:654-659
            terminate();
            ++iteration;
            break;
        }
        if (rate_hz > 0) {
            next += std::chrono::duration_cast<std::chrono::steady_clock::duration>(period);
            std::this_thread::sleep_until(next);
        }
    }
    return iteration;
}

long WholeBodyController::run() {
    // cpp:678-683: the control loop on its own thread, the callbacks on this one (ros::spin).
    // shutdown_ is not cleared here either (as controlLoop): a requestShutdown() from another thread
    // before run() is not dropped; resetShutdown() clears it for a new run
    std::atomic<bool> finished{false};
    std::exception_ptr err;
    long cycles = 0;
    const double rate = runRate_ < 0.0 ? params_.loop_rate : runRate_;
    std::thread ctrl([&]() {
        try {
            cycles = loop(LONG_MAX, rate, loopHook);
        } catch (...) {
            err = std::current_exception();
        }
        finished.store(true);
    });
    while (!finished.load()) {  // ros::spin(): returns once the node shuts down
        if (spinOnce) {
            try {
                spinOnce();
            } catch (...) {
                requestShutdown();
                ctrl.join();
                throw;
            }
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    ctrl.join();
    if (err) std::rethrow_exception(err);
    return cycles;
}

}  // namespace wbc_mi355x
