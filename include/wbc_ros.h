/* wbc_ros.h — batched ROS1 wire adapters for the engine's C-ABI.
 *
 * Host-only library (libwbc_ros.so, no HIP): B serialized ROS1 messages in, the engine's
 * wbc_set_state / wbc_set_reference arrays out (include/wbc.h), and the engine's outputs back to
 * B serialized messages.  Each decoder is the reference's subscriber callback over raw bytes:
 *
 *   wbc_ros_decode_reference    referenceCallback(WbcReferenceMsg)   cpp:150-185
 *   wbc_ros_decode_model_states floatingBaseStateCallback(ModelStates) cpp:187-230 (model by name)
 *   wbc_ros_decode_joint_state  jointStateCallback(JointState)       cpp:232-254 (joints by name)
 *   wbc_ros_decode_twist        MotionPlanner::input_callback(Twist) motion_planner.cpp:122-127
 *   wbc_ros_encode_float64_array  the torque / GRF publishers       cpp:558-576
 *   wbc_ros_encode_reference      the planner's ref_pub_.publish    motion_planner.cpp:131
 *
 * Message b lives at msgs[b] with msg_lens[b] bytes (decoders) or at out + b * stride (encoders;
 * each encoded message has the same length, returned in *msg_len).  Every call returns WBC_OK or a
 * negative WBC_ERR_*; on WBC_ERR_ARG, wbc_ros_last_error() names the robot and the field.
 * Switching flags are not part of any message: the engine caller latches them (wbc.h).
 */
#ifndef WBC_ROS_H
#define WBC_ROS_H

#include <stdint.h>

#include "wbc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* MD5 sum of a message type for the TCPROS connection header ("std_msgs/Float64MultiArray",
 * "sensor_msgs/JointState", "gazebo_msgs/ModelStates", "geometry_msgs/Twist",
 * "anymal_wbc/WbcReferenceMsg"); NULL for any other type. */
const char* wbc_ros_md5sum(const char* datatype);
const char* wbc_ros_last_error(void);

/* WbcReferenceMsg -> ref [B][54] (pose 6, vel 6, acc 6, swing pos 12, vel 12, acc 12) and contacts
 * [B] (bit i = footContacts[i]).  A field shorter than the reference reads is an error. */
int32_t wbc_ros_decode_reference(const uint8_t* const* msgs, const uint64_t* msg_lens, int32_t B,
                                 double* ref, uint8_t* contacts);
/* ModelStates -> base_pose [B][7] (px, py, pz, qx, qy, qz, qw) and nu[B][18] entries 0..5 (linear,
 * angular).  model_name NULL = "anymalModel" (params_controller.yaml:1). */
int32_t wbc_ros_decode_model_states(const uint8_t* const* msgs, const uint64_t* msg_lens, int32_t B,
                                    const char* model_name, double* base_pose, double* nu);
/* JointState -> qj [B][12] and nu[B][18] entries 6..17, in model order; joint_names: the 12 model
 * joint names (NULL = LH_HAA, LH_HFE, ..., RH_KFE). */
int32_t wbc_ros_decode_joint_state(const uint8_t* const* msgs, const uint64_t* msg_lens, int32_t B,
                                   const char* const* joint_names, double* qj, double* nu);
/* Twist -> cmd [B][3] = (linear.x, linear.y, angular.z), the planner's command (wbc_planner.h). */
int32_t wbc_ros_decode_twist(const uint8_t* const* msgs, const uint64_t* msg_lens, int32_t B, double* cmd);

/* rows [B][n] -> B Float64MultiArray messages (empty layout, as published at cpp:558-576), each
 * 12 + 8 n bytes.  stride >= that. */
int32_t wbc_ros_encode_float64_array(const double* rows, int32_t B, int32_t n, uint8_t* out, uint64_t stride,
                                     uint64_t* msg_len);
/* ref [B][54] + contacts [B] -> B WbcReferenceMsg messages, each 508 bytes. */
int32_t wbc_ros_encode_reference(const double* ref, const uint8_t* contacts, int32_t B, uint8_t* out,
                                 uint64_t stride, uint64_t* msg_len);

#ifdef __cplusplus
}
#endif

#endif
