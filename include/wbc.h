/*
 * wbc.h — C-ABI of the MI355X batched whole-body-control engine.
 *
 * Drop-in boundary for the per-cycle hot path of the reference's `WholeBodyController`
 * (include/anymal_wbc/whole_body_controller.hpp:35-171, src/whole_body_controller.cpp:256-577):
 *
 *   reference call (file:line)                                   -> C-ABI entry point
 *   WholeBodyController::WholeBodyController()  cpp:22-59         -> wbc_create
 *   WholeBodyController::~WholeBodyController() cpp:61-63         -> wbc_destroy
 *   loadParameters()                            cpp:122-148       -> wbc_params (wbc_default_params)
 *   ModelLoader::loadModelFromFile(urdf)        cpp:26-40         -> wbc_model (wbc_anymal_model)
 *   floatingBaseStateCallback/jointStateCallback cpp:187-254      -> wbc_set_state
 *   referenceCallback(WbcReferenceMsg)          cpp:150-185       -> wbc_set_reference
 *   setInitialState() + firstControllerIteration_ cpp:65-120,523  -> wbc_reset
 *   updateState()                               cpp:256-294       -> wbc_update
 *   solveQP() + computeJointTorques()           cpp:466-577       -> wbc_solve
 *   controlLoop() body (update; solve; torques) cpp:650-652       -> wbc_step (fused)
 *   jointTorquePub_/desiredGroundReactionForcesPub_ cpp:563,576   -> wbc_get_output
 *   qpReturnValue_ != SUCCESSFUL_RETURN          cpp:654           -> per-robot status[] (WBC_QP_*)
 *
 * Conventions
 *  - Everything is fp64.  Sizes are compile-time constants of the reference (hpp:27-32).
 *  - A handle owns B robots ("batch").  Host arrays are robot-major per quantity
 *    (array[b * width + k]); each quantity is its own array (struct of arrays).
 *  - Leg / joint order: LH, LF, RF, RH x (HAA, HFE, KFE) — the reference's model order
 *    (cpp:81,234,327-341).  Contact bit i of contacts[b] = footContacts_[i] (cpp:183).
 *  - base_pose[b] = (px, py, pz, qx, qy, qz, qw) as in gazebo_msgs/ModelStates.pose (cpp:209-218).
 *  - nu[b] = (v_lin world (3), omega world (3), qdot (12)) = [baseVel_; jointVel_] (cpp:228,287).
 *  - ref[b] = WbcReferenceMsg field order (msg/WbcReferenceMsg.msg:1-6): desiredComPose (6),
 *    desiredComVelocity (6), desiredComAcceleration (6), desiredSwingLegsPosition (12),
 *    desiredSwingLegsVelocity (12), desiredSwingLegsAcceleration (12).
 *  - switching[b] = isSwitchingFootState_ (cpp:176-184); the caller latches it (quirk A.7).
 *  - Every call returns WBC_OK (0) or a negative error; no exceptions cross the boundary.
 *  - A handle is used by one host thread.  Inputs are snapshotted when the step kernel reads
 *    them, which removes the reference's callback/control-thread race (cpp:499,681-682).
 */
#ifndef WBC_H
#define WBC_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WBC_NUM_LEGS 4
#define WBC_NUM_JOINTS 12
#define WBC_NUM_DOF 18
#define WBC_NV 42 /* qpNumberOfVariables, hpp:31 */
#define WBC_NC 70 /* qpNumberOfConstraints, hpp:32 */
#define WBC_POSE_LEN 7
#define WBC_NU_LEN 18
#define WBC_REF_LEN 54

/* One lumped rigid body hanging off a revolute joint (tools/gen_model.py). */
typedef struct wbc_link {
    double R[9];       /* parent body frame -> joint frame at q = 0, row-major */
    double p[3];       /* joint origin in the parent body frame */
    double axis[3];    /* joint axis in the joint (= child body) frame */
    double mass;
    double com[3];     /* child body frame */
    double inertia[9]; /* about the com, child body axes, row-major */
} wbc_link;

/* Lumped ANYmal model: replaces iDynTree::Model built from urdf/anymal.urdf (cpp:26-40). */
typedef struct wbc_model {
    double base_mass;
    double base_com[3];
    double base_inertia[9];
    wbc_link link[WBC_NUM_LEGS][3]; /* legs LH, LF, RF, RH; links after HAA, HFE, KFE */
    double foot[WBC_NUM_LEGS][3];   /* {LH,LF,RF,RH}_FOOT origin in the SHANK body frame */
    double total_mass;              /* model_.getTotalMass(), cpp:72 */
} wbc_model;

/* Controller parameters: config/params_controller.yaml:1-12, read at cpp:122-148. */
typedef struct wbc_params {
    double friction;     /* mu */
    double loop_rate;    /* Hz; finite-difference step 1/loop_rate (cpp:394) */
    double max_torque;   /* torque limit rows R3 (cpp:506,513) */
    double kp, kp_z, kd, ki;        /* wrench PD(I) gains (cpp:429-432) */
    double kp_swing, kd_swing;      /* swing-foot PD (cpp:449-450) */
    double slack_weight;            /* R block of slacks (cpp:476) */
    double initial_reference_pose[6];
    double gravity;                 /* gravityAcceleration, hpp:30 */
    int32_t max_wsr;                /* nWSR = 100 (cpp:517) */
    int32_t reserved;
} wbc_params;

/* API return codes. */
enum {
    WBC_OK = 0,
    WBC_ERR_ARG = -1,
    WBC_ERR_HIP = -2,
    WBC_ERR_STATE = -3,
    WBC_ERR_NO_DEVICE = -4
};

/* Per-robot QP status (status[] output); 0 mirrors qpOASES SUCCESSFUL_RETURN (cpp:654). */
enum {
    WBC_QP_OK = 0,
    WBC_QP_MAX_ITER = 1,   /* more than max_wsr working-set changes (nWSR exceeded; see iters below) */
    WBC_QP_INFEASIBLE = 2, /* constraints inconsistent */
    WBC_QP_NUMERIC = 3     /* non-finite input or factorisation breakdown */
};

/* Step flags. */
#define WBC_STATELESS 1u /* cold step: history = reset values; history is neither read nor written.
                          * Without it the step is stateful: finite-difference history, integral
                          * error and a QP hotstart from the previous working set (as qpOASES
                          * SQProblem::hotstart, src/whole_body_controller.cpp:531). */
#define WBC_DEBUG 2u     /* also write the per-robot debug record (wbc_get_debug) */
#define WBC_NO_X 4u      /* skip the x[42] output (tau, grf, status, iters are still written) */
#define WBC_SPLIT 8u     /* wbc_step / wbc_step_modes as the split kernels (update, then the general
                          * 24-variable or four-contact solve kernel: wbc_update + wbc_solve) */
#define WBC_TIMED 16u    /* wbc_step records HIP events around its kernels (wbc_last_kernel_ms) */
#define WBC_COLD 32u     /* stateful, but the QP starts cold (no hotstart from the previous working set) */
#define WBC_FUSED 64u    /* wbc_step as the one-robot-per-wave kernel of the general 24-variable method */
#define WBC_GROUP 128u   /* device-bound contact masks (wbc_bind_device_inputs): group the QPs by mask on
                          * the stream before the step (one small kernel), as the engine does on the
                          * host for masks it copies.  Same results either way; it pays when the masks
                          * are mixed (waves of one mask), not when they are all equal (a trot). */
#define WBC_RESIDENT 256u /* wbc_cycle only, B <= 4: the step stays resident on the GPU between cycles (one
                          * workgroup polling a pinned mailbox), so a cycle costs no kernel launch and no
                          * stream synchronisation (the B = 1 drop-in).  The resident wave
                          * ends after 100 ms without a cycle, or at any other call on the engine (which
                          * waits for it); the next WBC_RESIDENT cycle starts it again.  Same results as a
                          * plain wbc_cycle. */

/* Debug record layout (doubles per robot), written by update/step under WBC_DEBUG. */
enum {
    WBC_DBG_COM = 0,        /* c (3)                       getCenterOfMassPosition (cpp:260) */
    WBC_DBG_COMVEL = 3,     /* c-dot (3)                   getCenterOfMassVelocity (cpp:261) */
    WBC_DBG_POSE = 6,       /* currentPose_ (6)            cpp:264 */
    WBC_DBG_VC = 12,        /* centerOfMassVelocity_ (6)   cpp:261 */
    WBC_DBG_M = 18,         /* mass matrix 18x18 row-major cpp:266 */
    WBC_DBG_CNU = 342,      /* C(q,nu) nu (18)             cpp:544-551 */
    WBC_DBG_JFEET = 360,    /* foot Jacobians rows 0-2, 12x18 (LH,LF,RF,RH) cpp:327-341 */
    WBC_DBG_PFEET = 576,    /* foot positions (12)         cpp:344-362 */
    WBC_DBG_VFEET = 588,    /* foot velocities (12)        cpp:364-382 */
    WBC_DBG_MBARB = 600,    /* centroidMassMatrixBase_ 6x6 cpp:271 */
    WBC_DBG_MBARJ = 636,    /* centroidMassMatrixJoints_ 12x12 cpp:272 */
    WBC_DBG_JBAR = 780,     /* J_feet T^-1 (unmasked) 12x18 cpp:278-284 */
    WBC_DBG_BBAR = 996,     /* centroidGeneralizedBias_ (18) cpp:289 */
    WBC_DBG_WRENCH = 1014,  /* computeDesiredWrench (6)    cpp:426-445 */
    WBC_DBG_R1 = 1020,      /* R1 bounds: -Jc_dot v (12)   cpp:504 */
    WBC_DBG_RSW = 1032,     /* R4/R5 bound: cmd - Js_dot v (12) cpp:507,515 */
    WBC_DBG_STAMPS = 1044,  /* diagnostic builds only (-DWBC_STAMPS): s_memtime per phase (8) */
    WBC_DBG_LEN = 1052
};

typedef struct wbc_engine wbc_engine;

/* Defaults of config/params_controller.yaml and the lumped reference URDF. */
int32_t wbc_default_params(wbc_params* out);
int32_t wbc_anymal_model(wbc_model* out);
/* Model from a URDF file at run time (replaces ModelLoader::loadModelFromFile +
 * KinDynComputations::loadRobotModel, cpp:26-40, and the getFrameIndex lookups, cpp:327-379): any
 * 12-DoF quadruped whose legs are 3-revolute-joint chains off the floating base.  Fixed joints are
 * lumped into their parent bodies (exact for M, C nu and frame kinematics).  legs: the 4 leg name
 * prefixes in model order (NULL = LH, LF, RF, RH); joints: the 3 joint suffixes from the base out
 * (NULL = HAA, HFE, KFE), joint names <leg>_<suffix>; foot frames <leg>_<foot_suffix> (NULL = FOOT). */
int32_t wbc_model_from_urdf(const char* urdf_path, const char* const* legs, const char* const* joints,
                            const char* foot_suffix, wbc_model* out);

int32_t wbc_create(const wbc_model* model, const wbc_params* params, int32_t batch, int32_t device,
                   wbc_engine** out);
int32_t wbc_destroy(wbc_engine* h);
int32_t wbc_batch(const wbc_engine* h);
/* Use a caller-owned hipStream_t (NULL = the engine's own stream).  Work queued on the previous
 * stream is drained first (the call synchronizes it), so switching streams never races.  A bound
 * caller stream must stay alive until it is unbound (wbc_set_stream(h, NULL)) or the engine is
 * destroyed: both synchronize it.  (No event is recorded after each launch to track the stream:
 * its packet would cost ~3 us per step.) */
int32_t wbc_set_stream(wbc_engine* h, void* hip_stream);

/* Host inputs, copied to device on the engine stream. Any pointer may be NULL (= unchanged). */
int32_t wbc_set_state(wbc_engine* h, const double* base_pose, const double* nu, const double* qj);
int32_t wbc_set_reference(wbc_engine* h, const double* ref, const uint8_t* contacts,
                          const uint8_t* switching);
/* Device-resident inputs (no copy): the step reads these pointers directly.  NULL restores
 * the engine-owned buffer for that quantity. */
int32_t wbc_bind_device_inputs(wbc_engine* h, const double* d_base_pose, const double* d_nu,
                               const double* d_qj, const double* d_ref, const uint8_t* d_contacts,
                               const uint8_t* d_switching);

/* Caller-owned device output buffers (no copy): the step writes into these pointers directly
 * (e.g. a tensor that an RCCL all-gather then reads).  NULL restores the engine-owned buffer. */
int32_t wbc_bind_device_outputs(wbc_engine* h, double* d_tau, double* d_grf, double* d_x, int32_t* d_status,
                                int32_t* d_iters);

/* Reset robots to setInitialState() (cpp:65-120) + first-iteration cold start.  mask NULL = all. */
int32_t wbc_reset(wbc_engine* h, const uint8_t* mask);

/* updateState(): dynamics, centroidal transform, finite differences, assembly (stream-ordered). */
int32_t wbc_update(wbc_engine* h, uint32_t flags);
/* solveQP() + computeJointTorques() on the problem assembled by the last wbc_update. */
int32_t wbc_solve(wbc_engine* h, uint32_t flags);
/* update + solve + torques for one control cycle.  By default one kernel, four robots per wave:
 * each robot's QP is reduced exactly to 12 variables (the swing slacks and stance equalities
 * eliminated) and solved in place, any contact mask, stateless or stateful (with
 * the hotstart); a robot whose reduction is not usable (a near-singular stance leg) is solved with
 * the general 24-variable method by the same wave, inside the same launch (drain_fallbacks,
 * DESIGN.md 4.9).  A robot's result depends only on its own inputs, mask and flags, never on its
 * batch neighbours; the QPs are grouped by contact mask (one mask per wave: the host-copied masks'
 * map is built when they are copied, device-bound masks' under WBC_GROUP).
 * WBC_SPLIT: the update kernel then the solve kernels, the problem passing through HBM (the form
 * wbc_update + wbc_solve run); WBC_FUSED: one robot per wave, the general method with the problem
 * in LDS.  All forms return the same x and tau (to rounding) and the same status while the
 * working-set cap does not bind.  `iters` counts the working-set changes of the method that ran:
 * the 12-variable form's friction and torque rows by default, the general form's rows (the swing
 * slack rows included, the convention of a dense active set on the reference's 42 x 70 QP) under
 * WBC_SPLIT / WBC_FUSED.  WBC_QP_MAX_ITER is judged on that count against max_wsr, so near the cap
 * the default form (fewer changes for the same QP) can return WBC_QP_OK where the split / fused
 * forms return WBC_QP_MAX_ITER.
 * Every form picks the row to add as the most violated one by slack / |reference row|, with near-
 * ties treated as ties: the lowest row id among the rows within WBC_TIE_BAND (relative) of the
 * most violated, so the route (and `iters`) does not depend on rounding when two rows are violated
 * alike in exact arithmetic.  The C oracle (oracle/wbc_ref.c) applies the same rule.
 * The general form (WBC_SPLIT / WBC_FUSED and the default step's fallback) also treats an r_k (the
 * pending row's coefficient on active slot k) below WBC_R_REL times the largest |r| as zero, not as
 * a drop candidate: when the pending row depends on the active set (an infeasible QP), those r_k
 * are rounding noise, and the number of noise drops before WBC_QP_INFEASIBLE would otherwise
 * depend on the form's rounding. */
#define WBC_TIE_BAND 1e-9
#define WBC_R_REL 1e-12
int32_t wbc_step(wbc_engine* h, uint32_t flags);
int32_t wbc_synchronize(wbc_engine* h);

/* Contact-mode hypotheses (BASELINE configs[4]: every state solved under several contact masks).
 * After wbc_set_modes(h, K, modes) with K dividing the batch B, the engine holds S = B / K states:
 * wbc_set_state / wbc_set_reference / bound device inputs hold S rows (contacts[] is not read), and
 * wbc_step_modes solves K QPs per state: output row s * K + k is state s under contact mask
 * modes[k] (4-bit, footContacts_ order), bit-identical to a wbc_step on that state with
 * contacts = modes[k] (same flags).  By default each hypothesis runs in its own 16-lane segment
 * (the state's inputs read from L2 by its K segments, nothing through HBM); WBC_SPLIT computes the
 * dynamics and assembly (updateState, cpp:256-294) once per state and writes them to HBM for K
 * general solves.
 * Hypotheses are cold steps: flags must include WBC_STATELESS (WBC_DEBUG is refused).
 * wbc_update / wbc_solve / wbc_step return WBC_ERR_STATE while modes are set; K = 0 clears them. */
#define WBC_MAX_MODES 16
int32_t wbc_set_modes(wbc_engine* h, int32_t n_modes, const uint8_t* modes);
int32_t wbc_step_modes(wbc_engine* h, uint32_t flags);
/* Hypotheses per wave of the default wbc_step_modes (no reference counterpart; diagnostics): 1 =
 * one hypothesis per 16-lane segment (wbc_update_solve_kernel); M > 1 = the mode loop
 * (wbc_modes_kernel: one update per state and wave, then M hypotheses in turn), chosen by
 * wbc_set_modes from the batch and the device's CU count (WBC_MODES_M in the environment overrides
 * it with a divisor of n_modes).  Results are bit-identical either way. */
int32_t wbc_modes_per_wave(wbc_engine* h, int32_t* m);

/* One synchronous control cycle, host arrays in and out (the low-latency path for small batches,
 * e.g. the B = 1 drop-in of whole_body_controller_node): the inputs are packed into pinned staging
 * and sent in one H2D copy, the step runs (flags as wbc_step), and the outputs come back in one D2H
 * copy and one synchronize.  Same results as wbc_set_state + wbc_set_reference + wbc_step +
 * wbc_get_output.  Inputs are all required; any output may be NULL (x NULL also skips computing
 * it, as WBC_NO_X).  Input and output bindings (wbc_bind_device_*) are left as they were: the
 * cycle reads and writes the engine's own buffers for this one step.  Refused while mode
 * hypotheses are set. */
int32_t wbc_cycle(wbc_engine* h, const double* base_pose, const double* nu, const double* qj, const double* ref,
                  const uint8_t* contacts, const uint8_t* switching, uint32_t flags, double* tau, double* grf,
                  double* x, int32_t* status, int32_t* iters);

/* Outputs (host copies, synchronous).  Any pointer may be NULL.
 * tau [B][12], grf [B][12] (= x[18:30]), x [B][42], status [B], iters [B].
 * A robot whose status is not WBC_QP_OK gets tau, grf and x all zero (the reference publishes
 * qpOASES' last iterate and then stops its control loop, cpp:652-659; a batch keeps running, so
 * a failed robot publishes zeros instead of an unconverged iterate).  iters is the cap
 * (max_wsr) under WBC_QP_MAX_ITER. */
int32_t wbc_get_output(wbc_engine* h, double* tau, double* grf, double* x, int32_t* status,
                       int32_t* iters);
/* Device pointers of the output buffers (valid until wbc_destroy). */
int32_t wbc_device_outputs(wbc_engine* h, double** d_tau, double** d_grf, double** d_x,
                           int32_t** d_status, int32_t** d_iters);
/* Debug records [B][WBC_DBG_LEN] of the last update/step run with WBC_DEBUG. */
int32_t wbc_get_debug(wbc_engine* h, double* out);

/* Device time of the last wbc_step run with WBC_TIMED (ms, HIP events on the engine stream). */
int32_t wbc_last_kernel_ms(wbc_engine* h, double* ms);
const char* wbc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* WBC_H */
