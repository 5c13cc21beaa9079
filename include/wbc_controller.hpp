// wbc_controller.hpp — C++ host shim with the reference's WholeBodyController surface, backed by
// the MI355X engine (C-ABI in wbc.h), for the single-robot drop-in (B = 1).
//
// Reference surface (include/anymal_wbc/whole_body_controller.hpp:35-171):
//   WholeBodyController()                 hpp:38, cpp:22-59    -> WholeBodyController(params, device)
//   floatingBaseStateCallback(ModelStates) hpp:43, cpp:187-230 -> same name, ROS-free message struct
//   jointStateCallback(JointState)        hpp:44, cpp:232-254  -> same name, ROS-free message struct
//   referenceCallback(WbcReferenceMsg)    hpp:45, cpp:150-185  -> same name, ROS-free message struct
//   updateState()                         hpp:47, cpp:256-294  -> wbc_update
//   setInitialState()                     hpp:49, cpp:65-120   -> host state reset + wbc_reset
//   loadParameters()                      hpp:50, cpp:122-148  -> parameters passed to the constructor
//   solveQP()                             hpp:54, cpp:466-542  -> wbc_solve
//   computeJointTorques()                 hpp:52, cpp:553-577  -> wbc_get_output + publishers
//   controlLoop()                         hpp:67, cpp:637-676  -> controlLoop(max_iterations, ...)
//   run()                                 hpp:41, cpp:678-683  -> run(): control thread + spin
//   terminate()                           hpp:69, cpp:627-636  -> publishes zero torques
//
// ROS is absent here: messages are plain structs with the same field names, and publishers are
// std::function hooks.  The callbacks and the control cycle share the controller state under one
// mutex: a cycle copies the callback state under the lock and runs the engine outside it, so the
// callbacks may run on another thread (the reference shares that state with no synchronisation,
// cpp:681-682, and snapshots only jointVel_, cpp:499).
//
// The reference node (src/whole_body_controller_node.cpp:6-7) builds unchanged against this
// header: `WholeBodyController wbc; wbc.run();` (the class is also visible in the global
// namespace, below; define WBC_NO_GLOBAL_ALIAS to keep it in wbc_mi355x only).
#ifndef WBC_CONTROLLER_HPP
#define WBC_CONTROLLER_HPP

#include <array>
#include <atomic>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "wbc.h"

namespace wbc_mi355x {

constexpr int numberOfJoints = WBC_NUM_JOINTS;
constexpr int numberOfLegs = WBC_NUM_LEGS;
constexpr int qpNumberOfVariables = WBC_NV;

// std_msgs/Float64MultiArray, gazebo_msgs/ModelStates, sensor_msgs/JointState, anymal_wbc/WbcReferenceMsg
// (all fields of the ROS messages, so include/wbc_ros_wire.hpp round-trips their wire bytes)
struct MultiArrayDimension {
    std::string label;
    uint32_t size = 0, stride = 0;
};
struct MultiArrayLayout {
    std::vector<MultiArrayDimension> dim;
    uint32_t data_offset = 0;
};
struct Float64MultiArray {
    MultiArrayLayout layout;  // left empty by the reference (cpp:558-576)
    std::vector<double> data;
};
struct Time {
    uint32_t sec = 0, nsec = 0;
};
struct Header {
    uint32_t seq = 0;
    Time stamp;
    std::string frame_id;
};
struct Vector3 {
    double x = 0, y = 0, z = 0;
};
struct Quaternion {
    double x = 0, y = 0, z = 0, w = 1;
};
struct Pose {
    Vector3 position;
    Quaternion orientation;
};
struct Twist {
    Vector3 linear, angular;
};
struct ModelStates {
    std::vector<std::string> name;
    std::vector<Pose> pose;
    std::vector<Twist> twist;
};
struct JointState {
    Header header;
    std::vector<std::string> name;
    std::vector<double> position, velocity, effort;
};
struct WbcReferenceMsg {  // msg/WbcReferenceMsg.msg:1-7
    Float64MultiArray desiredComPose, desiredComVelocity, desiredComAcceleration;
    Float64MultiArray desiredSwingLegsPosition, desiredSwingLegsVelocity, desiredSwingLegsAcceleration;
    bool footContacts[numberOfLegs] = {true, true, true, true};
};

class WholeBodyController {
public:
    // model name matched in ModelStates.name (params_controller.yaml:1)
    static constexpr const char* modelName = "anymalModel";

    // params == nullptr: config/params_controller.yaml defaults.  Throws std::runtime_error if the
    // engine cannot be created (no HIP device, library error): there is no CPU fallback.
    explicit WholeBodyController(const wbc_params* params = nullptr, int device = 0);
    ~WholeBodyController();
    WholeBodyController(const WholeBodyController&) = delete;
    WholeBodyController& operator=(const WholeBodyController&) = delete;

    void floatingBaseStateCallback(const ModelStates& modelStateMsg);
    void jointStateCallback(const JointState& jointStateMsg);
    void referenceCallback(const WbcReferenceMsg& refMsg);

    void updateState();
    void setInitialState();
    void solveQP();
    void computeJointTorques();
    void terminate();
    // updateState(); solveQP(); computeJointTorques(); as one engine call (wbc_cycle: one H2D copy,
    // the step's kernels, one D2H copy, one synchronize) -- the body of controlLoop
    void controlCycle();
    // wbc_cycle flags for controlCycle.  Default WBC_RESIDENT: the step stays resident on the GPU
    // between cycles (no kernel launch and no stream synchronisation per cycle);
    // 0: a launch per cycle; WBC_FUSED: the one-robot-per-wave kernel
    void setStepFlags(uint32_t flags) { stepFlags_ = flags; }

    // ROS-free control loop (cpp:637-676): setInitialState, then per cycle
    //   beforeCycle(iteration) [stands in for the subscriber callbacks], controlCycle() (= updateState,
    //   solveQP, computeJointTorques); stops when the QP fails (cpp:654-659) or after max_iterations.
    // rate_hz > 0 sleeps to that rate like ros::Rate; 0 runs back to back.  Returns iterations run.
    // A requestShutdown() before or during the loop ends it (ros::ok() turns false and stays false,
    // cpp:648): the flag is not cleared on entry, so a shutdown requested before a control thread
    // reaches this call is not lost.  resetShutdown() clears it for a new loop.
    long controlLoop(long max_iterations, double rate_hz = 0.0,
                     const std::function<void(long)>& beforeCycle = nullptr);

    // run() (hpp:41, cpp:678-683): starts controlLoop on its own thread (boost::thread at cpp:681)
    // at params.loop_rate, and spins on the calling thread (ros::spin at cpp:682) until the loop
    // ends: the QP fails (cpp:654-659) or requestShutdown() is called (ros::ok() turns false).
    // While it spins it calls `spinOnce` repeatedly (the stand-in for ros::spin dispatching the
    // subscriber callbacks; a host's message source calls the *Callback methods from there or from
    // any other thread).  `loopHook(iteration)` runs on the control thread before every cycle.
    // Returns the cycles run.  Errors on the control thread (an engine failure) are rethrown here.
    // Like controlLoop, run() does not clear the shutdown flag on entry (a requestShutdown() from
    // another thread before run() ends it before its first cycle); resetShutdown() clears it.
    long run();
    void requestShutdown() { shutdown_.store(true); }
    void resetShutdown() { shutdown_.store(false); }
    bool ok() const { return !shutdown_.load(); }
    std::function<void()> spinOnce;
    std::function<void(long)> loopHook;
    // 0 runs the loop back to back (tests); default: params.loop_rate (400 Hz, cpp:639,673)
    void setRunRate(double rate_hz) { runRate_ = rate_hz; }

    // publishers (cpp:41-43): jointTorquePub_, desiredGroundReactionForcesPub_
    std::function<void(const Float64MultiArray&)> jointTorquePublisher;
    std::function<void(const Float64MultiArray&)> desiredGroundReactionForcesPublisher;

    // qpReturnValue_ (hpp:166): WBC_QP_OK mirrors qpOASES::SUCCESSFUL_RETURN
    int qpReturnValue() const { return qpStatus_; }
    int qpIterations() const { return qpIters_; }
    const std::array<double, numberOfJoints>& jointTorques() const { return tau_; }
    const std::array<double, 3 * numberOfLegs>& groundReactionForces() const { return grf_; }
    const std::array<double, qpNumberOfVariables>& qpSolution() const { return x_; }
    bool isSwitchingFootState() const { return isSwitchingFootState_; }
    wbc_engine* engine() { return engine_; }

private:
    struct Inputs {  // the callback state one cycle uses, copied under mu_
        double basePose[WBC_POSE_LEN];
        double nu[WBC_NU_LEN];
        double jointPos[numberOfJoints];
        double ref[WBC_REF_LEN];
        uint8_t contacts;
        uint8_t switching;
    };
    Inputs snapshot();
    void pushInputs();
    void publish();

    std::mutex mu_;  // callbacks vs the control cycle's snapshot
    std::atomic<bool> shutdown_{false};
    // the loop itself; run() calls it without clearing shutdown_, so a requestShutdown() issued
    // between run()'s start and the control thread's first cycle is not lost
    long loop(long max_iterations, double rate_hz, const std::function<void(long)>& beforeCycle);
    double runRate_ = -1.0;  // < 0: params_.loop_rate

    wbc_engine* engine_ = nullptr;
    wbc_params params_{};
    bool firstJointStateCallback_ = true;
    bool firstFloatingBaseStateCallback_ = true;
    bool firstControllerIteration_ = true;
    int modelIndex_ = 0;
    int jointIndex_[numberOfJoints] = {};

    // state (cpp:65-120 initial values)
    double basePose_[WBC_POSE_LEN] = {};  // px py pz qx qy qz qw
    double nu_[WBC_NU_LEN] = {};           // v_lin, omega (world), qdot
    double jointPos_[numberOfJoints] = {};
    double ref_[WBC_REF_LEN] = {};          // WbcReferenceMsg field order
    int footContacts_[numberOfLegs] = {1, 1, 1, 1};
    bool isSwitchingFootState_ = false;

    // one robot, per control cycle (profiles/r05/b1_*.log, mean / p99): the resident step
    // (WBC_RESIDENT) 26.1 / 26.3 us, a launch per cycle (0) 34.0 / 37.8 us, WBC_FUSED (one robot
    // per wave, the 24-variable form) 39.3 / 43.4 us
    uint32_t stepFlags_ = WBC_RESIDENT;
    int qpStatus_ = WBC_QP_OK;
    int qpIters_ = 0;
    std::array<double, numberOfJoints> tau_{};
    std::array<double, 3 * numberOfLegs> grf_{};
    std::array<double, qpNumberOfVariables> x_{};
};

// The reference model's joint names in model order (LH, LF, RF, RH x HAA, HFE, KFE), used to map
// JointState messages by name (cpp:234-246).
const std::array<std::string, numberOfJoints>& modelJointNames();

}  // namespace wbc_mi355x

#ifndef WBC_NO_GLOBAL_ALIAS
// the name the reference node uses (src/whole_body_controller_node.cpp:6)
using wbc_mi355x::WholeBodyController;
#endif

#endif  // WBC_CONTROLLER_HPP
