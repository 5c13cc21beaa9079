// wbc_ros_wire.hpp — ROS1 wire format (TCPROS / rosbag message bytes) for the shim's message
// structs (include/wbc_controller.hpp), SURVEY.md §8(f) rank 4.
//
// The reference talks to the rest of the system only through ROS1 topics
// (src/whole_body_controller.cpp:42-49): it subscribes to gazebo_msgs/ModelStates,
// sensor_msgs/JointState and anymal_wbc/WbcReferenceMsg (msg/WbcReferenceMsg.msg:1-7) and
// publishes std_msgs/Float64MultiArray torques and ground reaction forces (cpp:558-576); the
// motion planner subscribes to geometry_msgs/Twist on /cmd_vel (src/motion_planner.cpp:122-130).
// These functions turn the exact bytes roscpp puts on the wire (or rosbag stores) into the shim's
// structs and back, so a bridge (topic_tools::ShapeShifter, a rosbag reader, a raw TCPROS socket)
// can feed the MI355X controller without linking roscpp.
//
// ROS1 serialization: little-endian; string = uint32 length + bytes; variable array = uint32
// count + elements; fixed array (bool[4]) = elements only; bool = uint8; time = uint32 sec,
// uint32 nsec.  Decoders throw std::runtime_error on truncated or malformed input and return the
// number of bytes consumed.
#ifndef WBC_ROS_WIRE_HPP
#define WBC_ROS_WIRE_HPP

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "wbc_controller.hpp"

namespace wbc_mi355x {
namespace ros_wire {

// ros::message_traits::DataType / MD5Sum for each message (the TCPROS connection header fields)
template <class M> struct Traits;
template <> struct Traits<Float64MultiArray> {
    static constexpr const char* datatype = "std_msgs/Float64MultiArray";
    static constexpr const char* md5sum = "4b7d974086d4060e7db4613a7e6c3ba4";
};
template <> struct Traits<JointState> {
    static constexpr const char* datatype = "sensor_msgs/JointState";
    static constexpr const char* md5sum = "3066dcd76a6cfaef579bd0f34173e9fd";
};
template <> struct Traits<ModelStates> {
    static constexpr const char* datatype = "gazebo_msgs/ModelStates";
    static constexpr const char* md5sum = "48c080191eb15c41858319b4d8a609c2";
};
template <> struct Traits<Twist> {
    static constexpr const char* datatype = "geometry_msgs/Twist";
    static constexpr const char* md5sum = "9f195f881246fdfa2798d1d3eebca84a";
};
template <> struct Traits<WbcReferenceMsg> {
    static constexpr const char* datatype = "anymal_wbc/WbcReferenceMsg";
    static constexpr const char* md5sum = "422e395754f817c54d30baf1df2acdc2";  // checked in tests
};

// Append the serialized message to `out`.
void serialize(const Float64MultiArray& m, std::vector<uint8_t>& out);
void serialize(const JointState& m, std::vector<uint8_t>& out);
void serialize(const ModelStates& m, std::vector<uint8_t>& out);
void serialize(const Twist& m, std::vector<uint8_t>& out);
void serialize(const WbcReferenceMsg& m, std::vector<uint8_t>& out);

// Decode one message from buf[0, len); returns the bytes consumed.
size_t deserialize(const uint8_t* buf, size_t len, Float64MultiArray& m);
size_t deserialize(const uint8_t* buf, size_t len, JointState& m);
size_t deserialize(const uint8_t* buf, size_t len, ModelStates& m);
size_t deserialize(const uint8_t* buf, size_t len, Twist& m);
size_t deserialize(const uint8_t* buf, size_t len, WbcReferenceMsg& m);

template <class M> std::vector<uint8_t> serialize(const M& m) {
    std::vector<uint8_t> v;
    serialize(m, v);
    return v;
}

}  // namespace ros_wire
}  // namespace wbc_mi355x

#endif
