// wbc_ros_wire.cpp — ROS1 message bytes <-> shim structs (include/wbc_ros_wire.hpp) and the
// batched C-ABI over them (include/wbc_ros.h).  Host-only: no HIP, no roscpp.
#include "wbc_ros_wire.hpp"

#include <cstring>
#include <stdexcept>
#include <string>

#include "wbc_ros.h"

namespace wbc_mi355x {
namespace ros_wire {

namespace {

// ---------------------------------------------------------------- writer (little-endian host)
struct Writer {
    std::vector<uint8_t>& out;
    void raw(const void* p, size_t n) {
        const auto* b = static_cast<const uint8_t*>(p);
        out.insert(out.end(), b, b + n);
    }
    void u8(uint8_t v) { out.push_back(v); }
    void u32(uint32_t v) { raw(&v, 4); }
    void f64(double v) { raw(&v, 8); }
    void str(const std::string& s) {
        u32((uint32_t)s.size());
        raw(s.data(), s.size());
    }
    void f64s(const std::vector<double>& v) {
        u32((uint32_t)v.size());
        raw(v.data(), v.size() * 8);
    }
    void vec3(const Vector3& v) { f64(v.x); f64(v.y); f64(v.z); }
};

// ---------------------------------------------------------------- reader (bounds-checked)
struct Reader {
    const uint8_t* p;
    size_t n, at = 0;
    const char* what;
    void need(size_t k) {
        if (k > n - at) throw std::runtime_error(std::string(what) + ": truncated message");
    }
    void raw(void* dst, size_t k) {
        need(k);
        std::memcpy(dst, p + at, k);
        at += k;
    }
    uint8_t u8() { uint8_t v; raw(&v, 1); return v; }
    uint32_t u32() { uint32_t v; raw(&v, 4); return v; }
    double f64() { double v; raw(&v, 8); return v; }
    uint32_t count(size_t elem_bytes) {  // array length, checked against the bytes left
        const uint32_t c = u32();
        if (elem_bytes && (uint64_t)c * elem_bytes > n - at)
            throw std::runtime_error(std::string(what) + ": array length beyond the message");
        return c;
    }
    std::string str() {
        const uint32_t k = count(1);
        std::string s(reinterpret_cast<const char*>(p + at), k);
        at += k;
        return s;
    }
    std::vector<double> f64s() {
        const uint32_t c = count(8);
        std::vector<double> v(c);
        raw(v.data(), (size_t)c * 8);
        return v;
    }
    Vector3 vec3() { Vector3 v; v.x = f64(); v.y = f64(); v.z = f64(); return v; }
};

void put(Writer& w, const Float64MultiArray& m) {
    w.u32((uint32_t)m.layout.dim.size());
    for (const auto& d : m.layout.dim) { w.str(d.label); w.u32(d.size); w.u32(d.stride); }
    w.u32(m.layout.data_offset);
    w.f64s(m.data);
}

void get(Reader& r, Float64MultiArray& m) {
    const uint32_t nd = r.count(12);  // label length + size + stride
    m.layout.dim.resize(nd);
    for (auto& d : m.layout.dim) { d.label = r.str(); d.size = r.u32(); d.stride = r.u32(); }
    m.layout.data_offset = r.u32();
    m.data = r.f64s();
}

template <class M>  // WbcReferenceMsg or const WbcReferenceMsg
auto ref_fields(M& m, int k) -> decltype(&m.desiredComPose) {
    decltype(&m.desiredComPose) f[6] = {&m.desiredComPose, &m.desiredComVelocity, &m.desiredComAcceleration,
                               &m.desiredSwingLegsPosition, &m.desiredSwingLegsVelocity,
                               &m.desiredSwingLegsAcceleration};
    return f[k];
}

}  // namespace

// ---------------------------------------------------------------- per-message serializers
void serialize(const Float64MultiArray& m, std::vector<uint8_t>& out) {
    Writer w{out};
    put(w, m);
}

void serialize(const JointState& m, std::vector<uint8_t>& out) {
    Writer w{out};
    w.u32(m.header.seq); w.u32(m.header.stamp.sec); w.u32(m.header.stamp.nsec); w.str(m.header.frame_id);
    w.u32((uint32_t)m.name.size());
    for (const auto& s : m.name) w.str(s);
    w.f64s(m.position); w.f64s(m.velocity); w.f64s(m.effort);
}

void serialize(const ModelStates& m, std::vector<uint8_t>& out) {
    Writer w{out};
    w.u32((uint32_t)m.name.size());
    for (const auto& s : m.name) w.str(s);
    w.u32((uint32_t)m.pose.size());
    for (const auto& p : m.pose) {
        w.vec3(p.position);
        w.f64(p.orientation.x); w.f64(p.orientation.y); w.f64(p.orientation.z); w.f64(p.orientation.w);
    }
    w.u32((uint32_t)m.twist.size());
    for (const auto& t : m.twist) { w.vec3(t.linear); w.vec3(t.angular); }
}

void serialize(const Twist& m, std::vector<uint8_t>& out) {
    Writer w{out};
    w.vec3(m.linear); w.vec3(m.angular);
}

void serialize(const WbcReferenceMsg& m, std::vector<uint8_t>& out) {
    Writer w{out};
    for (int k = 0; k < 6; ++k) put(w, *ref_fields(m, k));
    for (int i = 0; i < numberOfLegs; ++i) w.u8(m.footContacts[i] ? 1 : 0);  // bool[4]: no length prefix
}

// ---------------------------------------------------------------- per-message deserializers
size_t deserialize(const uint8_t* buf, size_t len, Float64MultiArray& m) {
    Reader r{buf, len, 0, "Float64MultiArray"};
    get(r, m);
    return r.at;
}

size_t deserialize(const uint8_t* buf, size_t len, JointState& m) {
    Reader r{buf, len, 0, "JointState"};
    m.header.seq = r.u32(); m.header.stamp.sec = r.u32(); m.header.stamp.nsec = r.u32();
    m.header.frame_id = r.str();
    m.name.resize(r.count(4));
    for (auto& s : m.name) s = r.str();
    m.position = r.f64s(); m.velocity = r.f64s(); m.effort = r.f64s();
    return r.at;
}

size_t deserialize(const uint8_t* buf, size_t len, ModelStates& m) {
    Reader r{buf, len, 0, "ModelStates"};
    m.name.resize(r.count(4));
    for (auto& s : m.name) s = r.str();
    m.pose.resize(r.count(56));
    for (auto& p : m.pose) {
        p.position = r.vec3();
        p.orientation.x = r.f64(); p.orientation.y = r.f64(); p.orientation.z = r.f64(); p.orientation.w = r.f64();
    }
    m.twist.resize(r.count(48));
    for (auto& t : m.twist) { t.linear = r.vec3(); t.angular = r.vec3(); }
    return r.at;
}

size_t deserialize(const uint8_t* buf, size_t len, Twist& m) {
    Reader r{buf, len, 0, "Twist"};
    m.linear = r.vec3(); m.angular = r.vec3();
    return r.at;
}

size_t deserialize(const uint8_t* buf, size_t len, WbcReferenceMsg& m) {
    Reader r{buf, len, 0, "WbcReferenceMsg"};
    for (int k = 0; k < 6; ++k) get(r, *ref_fields(m, k));
    for (int i = 0; i < numberOfLegs; ++i) m.footContacts[i] = r.u8() != 0;
    return r.at;
}

}  // namespace ros_wire
}  // namespace wbc_mi355x

// ==================================================================== batched C-ABI (wbc_ros.h)
using namespace wbc_mi355x;

namespace {

thread_local std::string g_err;

int32_t fail(int32_t b, const std::string& what) {
    g_err = "robot " + std::to_string(b) + ": " + what;
    return WBC_ERR_ARG;
}

constexpr const char* kModelJointNames[numberOfJoints] = {
    "LH_HAA", "LH_HFE", "LH_KFE", "LF_HAA", "LF_HFE", "LF_KFE",
    "RF_HAA", "RF_HFE", "RF_KFE", "RH_HAA", "RH_HFE", "RH_KFE"};

// Decode B messages of type M and hand each to fn(b, msg); exceptions become WBC_ERR_ARG.
template <class M, class F>
int32_t decode_batch(const uint8_t* const* msgs, const uint64_t* lens, int32_t B, F&& fn) {
    if (B < 0 || (B > 0 && (!msgs || !lens))) return fail(-1, "null message array");
    M m;
    for (int32_t b = 0; b < B; ++b) {
        if (!msgs[b]) return fail(b, "null message");
        try {
            ros_wire::deserialize(msgs[b], (size_t)lens[b], m);
            fn(b, m);
        } catch (const std::exception& e) {
            return fail(b, e.what());
        }
    }
    return WBC_OK;
}

}  // namespace

extern "C" {

const char* wbc_ros_last_error(void) { return g_err.c_str(); }

const char* wbc_ros_md5sum(const char* datatype) {
    if (!datatype) return nullptr;
    const struct { const char *t, *m; } tab[] = {
        {ros_wire::Traits<Float64MultiArray>::datatype, ros_wire::Traits<Float64MultiArray>::md5sum},
        {ros_wire::Traits<JointState>::datatype, ros_wire::Traits<JointState>::md5sum},
        {ros_wire::Traits<ModelStates>::datatype, ros_wire::Traits<ModelStates>::md5sum},
        {ros_wire::Traits<Twist>::datatype, ros_wire::Traits<Twist>::md5sum},
        {ros_wire::Traits<WbcReferenceMsg>::datatype, ros_wire::Traits<WbcReferenceMsg>::md5sum}};
    for (const auto& e : tab)
        if (std::strcmp(e.t, datatype) == 0) return e.m;
    return nullptr;
}

int32_t wbc_ros_decode_reference(const uint8_t* const* msgs, const uint64_t* lens, int32_t B, double* ref,
                                 uint8_t* contacts) {
    if (B > 0 && (!ref || !contacts)) return fail(-1, "null output");
    return decode_batch<WbcReferenceMsg>(msgs, lens, B, [&](int32_t b, WbcReferenceMsg& m) {
        // referenceCallback, cpp:150-175: the first 6/6/6/12/12/12 entries of each field
        static const int n[6] = {6, 6, 6, 12, 12, 12};
        static const char* names[6] = {"desiredComPose", "desiredComVelocity", "desiredComAcceleration",
                                       "desiredSwingLegsPosition", "desiredSwingLegsVelocity",
                                       "desiredSwingLegsAcceleration"};
        const Float64MultiArray* f[6] = {&m.desiredComPose, &m.desiredComVelocity, &m.desiredComAcceleration,
                                         &m.desiredSwingLegsPosition, &m.desiredSwingLegsVelocity,
                                         &m.desiredSwingLegsAcceleration};
        double* r = ref + (size_t)b * WBC_REF_LEN;
        for (int k = 0, off = 0; k < 6; off += n[k], ++k) {
            if ((int)f[k]->data.size() < n[k])
                throw std::runtime_error(std::string(names[k]) + " has " + std::to_string(f[k]->data.size()) +
                                         " entries, " + std::to_string(n[k]) + " needed");
            std::memcpy(r + off, f[k]->data.data(), n[k] * sizeof(double));
        }
        uint8_t c = 0;  // cpp:176-184
        for (int i = 0; i < numberOfLegs; ++i) c |= (uint8_t)(m.footContacts[i] ? 1u << i : 0u);
        contacts[b] = c;
    });
}

int32_t wbc_ros_decode_model_states(const uint8_t* const* msgs, const uint64_t* lens, int32_t B,
                                    const char* model_name, double* base_pose, double* nu) {
    if (B > 0 && (!base_pose || !nu)) return fail(-1, "null output");
    const std::string want = model_name ? model_name : "anymalModel";
    return decode_batch<ModelStates>(msgs, lens, B, [&](int32_t b, ModelStates& m) {
        size_t k = 0;  // cpp:189-204: the model is located by name
        while (k < m.name.size() && m.name[k] != want) ++k;
        if (k == m.name.size() || k >= m.pose.size() || k >= m.twist.size())
            throw std::runtime_error("model '" + want + "' not in ModelStates");
        const Pose& p = m.pose[k];  // cpp:207-227
        const Twist& t = m.twist[k];
        double* q = base_pose + (size_t)b * 7;
        q[0] = p.position.x; q[1] = p.position.y; q[2] = p.position.z;
        q[3] = p.orientation.x; q[4] = p.orientation.y; q[5] = p.orientation.z; q[6] = p.orientation.w;
        double* v = nu + (size_t)b * WBC_NU_LEN;
        v[0] = t.linear.x; v[1] = t.linear.y; v[2] = t.linear.z;
        v[3] = t.angular.x; v[4] = t.angular.y; v[5] = t.angular.z;
    });
}

int32_t wbc_ros_decode_joint_state(const uint8_t* const* msgs, const uint64_t* lens, int32_t B,
                                   const char* const* joint_names, double* qj, double* nu) {
    if (B > 0 && (!qj || !nu)) return fail(-1, "null output");
    const char* const* names = joint_names ? joint_names : kModelJointNames;
    return decode_batch<JointState>(msgs, lens, B, [&](int32_t b, JointState& m) {
        for (int i = 0; i < numberOfJoints; ++i) {  // cpp:234-253: model order by name
            size_t k = 0;
            while (k < m.name.size() && m.name[k] != names[i]) ++k;
            if (k == m.name.size()) throw std::runtime_error(std::string("joint ") + names[i] + " not in JointState");
            if (k >= m.position.size() || k >= m.velocity.size())
                throw std::runtime_error(std::string("joint ") + names[i] + " has no position/velocity");
            qj[(size_t)b * numberOfJoints + i] = m.position[k];
            nu[(size_t)b * WBC_NU_LEN + 6 + i] = m.velocity[k];
        }
    });
}

int32_t wbc_ros_decode_twist(const uint8_t* const* msgs, const uint64_t* lens, int32_t B, double* cmd) {
    if (B > 0 && !cmd) return fail(-1, "null output");
    return decode_batch<Twist>(msgs, lens, B, [&](int32_t b, Twist& m) {
        double* c = cmd + (size_t)b * 3;  // motion_planner.cpp:122-126
        c[0] = m.linear.x; c[1] = m.linear.y; c[2] = m.angular.z;
    });
}

int32_t wbc_ros_encode_float64_array(const double* rows, int32_t B, int32_t n, uint8_t* out, uint64_t stride,
                                     uint64_t* msg_len) {
    const uint64_t len = 12 + 8ull * (uint64_t)(n < 0 ? 0 : n);
    if (msg_len) *msg_len = len;
    if (B < 0 || n < 0) return fail(-1, "negative size");
    if (B == 0) return WBC_OK;
    if (!rows || !out) return fail(-1, "null buffer");
    if (stride < len) return fail(-1, "stride " + std::to_string(stride) + " < message length " + std::to_string(len));
    for (int32_t b = 0; b < B; ++b) {
        uint8_t* o = out + (size_t)b * stride;
        const uint32_t hdr[3] = {0u, 0u, (uint32_t)n};  // dim[] empty, data_offset 0, data length
        std::memcpy(o, hdr, 12);
        std::memcpy(o + 12, rows + (size_t)b * n, 8 * (size_t)n);
    }
    return WBC_OK;
}

int32_t wbc_ros_encode_reference(const double* ref, const uint8_t* contacts, int32_t B, uint8_t* out,
                                 uint64_t stride, uint64_t* msg_len) {
    static const int n[6] = {6, 6, 6, 12, 12, 12};
    const uint64_t len = 6 * 12 + 8 * WBC_REF_LEN + numberOfLegs;  // 508
    if (msg_len) *msg_len = len;
    if (B < 0) return fail(-1, "negative size");
    if (B == 0) return WBC_OK;
    if (!ref || !contacts || !out) return fail(-1, "null buffer");
    if (stride < len) return fail(-1, "stride " + std::to_string(stride) + " < message length " + std::to_string(len));
    for (int32_t b = 0; b < B; ++b) {
        uint8_t* o = out + (size_t)b * stride;
        const double* r = ref + (size_t)b * WBC_REF_LEN;
        for (int k = 0; k < 6; ++k) {
            const uint32_t hdr[3] = {0u, 0u, (uint32_t)n[k]};
            std::memcpy(o, hdr, 12);
            std::memcpy(o + 12, r, 8 * (size_t)n[k]);
            o += 12 + 8 * n[k];
            r += n[k];
        }
        for (int i = 0; i < numberOfLegs; ++i) o[i] = (uint8_t)((contacts[b] >> i) & 1u);
    }
    return WBC_OK;
}

}  // extern "C"
