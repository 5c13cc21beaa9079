/*
 * wbc_planner.h — batched motion planner (the reference's MotionPlanner, one robot per thread).
 *
 * produces the WbcReferenceMsg task references (quintic CoM segment,
 * cubic Bezier swing feet, contact schedule LH -> RH -> LF -> RF) for B robots on the GPU, written
 * straight into device buffers that the WBC engine reads (wbc_bind_device_inputs), so an RL-style
 * batch needs no host -> device reference traffic.
 *
 *   reference (file:line)                                        -> C-ABI
 *   MotionPlanner::MotionPlanner()          src/motion_planner.cpp:129-168 -> wbc_planner_create / _reset
 *   MotionPlanner::load_parameters()        cpp:99-120, config/params_planner.yaml -> wbc_planner_params
 *   MotionPlanner::input_callback(Twist)    cpp:122-127          -> wbc_planner_set_command
 *   one ros::Rate tick of plannerLoop()     cpp:171-376          -> wbc_planner_tick
 *   ref_pub_.publish(ref_msg_)              cpp:338, 368         -> the device reference buffers
 *
 * A tick is one `rate.sleep()` of plannerLoop (dt = 0.01 s).  Ticks that publish nothing in the
 * reference (the step-phase transitions and the sleep after each 4-step cycle) leave the output
 * buffers unchanged and report published[b] = 0, so the engine keeps the last message, as the
 * reference controller keeps its last received reference.  switching[b] is set on publication when
 * the contacts differ from the previous published message: referenceCallback's
 * isSwitchingFootState_ (src/whole_body_controller.cpp:176-184), initial contacts 1111.
 */
#ifndef WBC_PLANNER_H
#define WBC_PLANNER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wbc_planner_params {  /* config/params_planner.yaml:1-8 */
    double step_length;
    double height_control_point;
    double x_offset;
    double y_offset;
    double step_duration;
    double body_height;
    double body_initial_velocity; /* read by load_parameters (cpp:114), absent from the YAML, unused */
    double body_final_velocity;
    double dt;
} wbc_planner_params;

typedef struct wbc_planner wbc_planner;

int32_t wbc_planner_default_params(wbc_planner_params* out);
int32_t wbc_planner_create(const wbc_planner_params* params, int32_t batch, int32_t device, wbc_planner** out);
int32_t wbc_planner_destroy(wbc_planner* p);
int32_t wbc_planner_set_stream(wbc_planner* p, void* hip_stream);
/* cmd[b] = (linear.x, linear.y, angular.z) of /cmd_vel (input_callback); host array [B][3] */
int32_t wbc_planner_set_command(wbc_planner* p, const double* cmd);
/* back to the constructor state (cpp:129-168); mask NULL = all robots */
int32_t wbc_planner_reset(wbc_planner* p, const uint8_t* mask);
/* advance every robot by one planner tick (stream-ordered) */
int32_t wbc_planner_tick(wbc_planner* p);
/* device outputs: ref [B][54] (WbcReferenceMsg field order, as wbc_set_reference), contacts [B]
 * (bit i = leg i, LH LF RF RH), switching [B], published [B] (1 if this tick published) */
int32_t wbc_planner_device_outputs(wbc_planner* p, double** ref, uint8_t** contacts, uint8_t** switching,
                                   uint8_t** published);
/* host copies of the same (synchronous); any pointer may be NULL */
int32_t wbc_planner_get_output(wbc_planner* p, double* ref, uint8_t* contacts, uint8_t* switching,
                               uint8_t* published);

#ifdef __cplusplus
}
#endif
#endif /* WBC_PLANNER_H */
