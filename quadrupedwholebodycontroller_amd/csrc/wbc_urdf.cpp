// wbc_urdf.cpp — URDF -> wbc_model at run time.
//
// Replaces the reference's iDynTree::ModelLoader::loadModelFromFile + KinDynComputations::
// loadRobotModel (src/whole_body_controller.cpp:26-40) and getFrameIndex lookups (cpp:327-379)
// for any 12-DoF quadruped: every fixed joint is lumped into its parent body (exact for mass
// matrix, bias forces and frame kinematics), the three revolute joints of each leg are found by
// name, and the foot frame is located by name inside the last body.  Same algorithm as
// tools/gen_model.py (which produced the committed ANYmal constants).  A small XML reader is
// included: URDF needs elements and attributes only.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "wbc.h"

extern "C" void wbc_internal_set_error(const char* msg);

namespace {

struct Xml {
    std::string name;
    std::map<std::string, std::string> attr;
    std::vector<std::unique_ptr<Xml>> kids;
    const Xml* child(const char* n) const {
        for (const auto& k : kids)
            if (k->name == n) return k.get();
        return nullptr;
    }
    std::string get(const char* a, const char* def = "") const {
        auto it = attr.find(a);
        return it == attr.end() ? std::string(def) : it->second;
    }
};

// elements, attributes, comments, processing instructions, CDATA-free text (ignored)
bool parse_xml(const std::string& s, Xml& root, std::string& err) {
    std::vector<Xml*> stack{&root};
    size_t i = 0;
    auto ws = [&](size_t& k) { while (k < s.size() && isspace((unsigned char)s[k])) ++k; };
    while (i < s.size()) {
        const size_t lt = s.find('<', i);
        if (lt == std::string::npos) break;
        if (s.compare(lt, 4, "<!--") == 0) {
            const size_t e = s.find("-->", lt + 4);
            if (e == std::string::npos) { err = "unterminated comment"; return false; }
            i = e + 3;
            continue;
        }
        if (s.compare(lt, 2, "<?") == 0 || s.compare(lt, 2, "<!") == 0) {
            const size_t e = s.find('>', lt);
            if (e == std::string::npos) { err = "unterminated declaration"; return false; }
            i = e + 1;
            continue;
        }
        if (s.compare(lt, 2, "</") == 0) {
            const size_t e = s.find('>', lt);
            if (e == std::string::npos || stack.size() < 2) { err = "bad closing tag"; return false; }
            stack.pop_back();
            i = e + 1;
            continue;
        }
        size_t k = lt + 1;
        const size_t n0 = k;
        while (k < s.size() && !isspace((unsigned char)s[k]) && s[k] != '>' && s[k] != '/') ++k;
        auto el = std::make_unique<Xml>();
        el->name = s.substr(n0, k - n0);
        bool self_close = false;
        for (;;) {
            ws(k);
            if (k >= s.size()) { err = "unterminated tag <" + el->name; return false; }
            if (s[k] == '/') { self_close = true; ++k; continue; }
            if (s[k] == '>') { ++k; break; }
            const size_t a0 = k;
            while (k < s.size() && s[k] != '=' && !isspace((unsigned char)s[k]) && s[k] != '>') ++k;
            const std::string an = s.substr(a0, k - a0);
            ws(k);
            if (k >= s.size() || s[k] != '=') { err = "attribute without value in <" + el->name; return false; }
            ++k;
            ws(k);
            if (k >= s.size() || (s[k] != '"' && s[k] != '\'')) { err = "unquoted attribute"; return false; }
            const char q = s[k++];
            const size_t v0 = k;
            while (k < s.size() && s[k] != q) ++k;
            el->attr[an] = s.substr(v0, k - v0);
            ++k;
        }
        Xml* raw = el.get();
        stack.back()->kids.push_back(std::move(el));
        if (!self_close) stack.push_back(raw);
        i = k;
    }
    if (stack.size() != 1) { err = "unclosed element <" + stack.back()->name; return false; }
    return true;
}

struct M3 {
    double a[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
};
struct V3 {
    double v[3] = {0, 0, 0};
};
M3 mul(const M3& A, const M3& B) {
    M3 C;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C.a[3 * i + j] = A.a[3 * i] * B.a[j] + A.a[3 * i + 1] * B.a[3 + j] + A.a[3 * i + 2] * B.a[6 + j];
    return C;
}
V3 mv(const M3& A, const V3& x) {
    V3 y;
    for (int i = 0; i < 3; ++i) y.v[i] = A.a[3 * i] * x.v[0] + A.a[3 * i + 1] * x.v[1] + A.a[3 * i + 2] * x.v[2];
    return y;
}
V3 add(const V3& a, const V3& b) { return V3{{a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]}}; }
M3 transpose(const M3& A) {
    M3 T;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T.a[3 * i + j] = A.a[3 * j + i];
    return T;
}
M3 rpy(double r, double p, double y) {  // URDF: R = Rz(yaw) Ry(pitch) Rx(roll)
    M3 Rx, Ry, Rz;
    Rx.a[4] = cos(r); Rx.a[5] = -sin(r); Rx.a[7] = sin(r); Rx.a[8] = cos(r);
    Ry.a[0] = cos(p); Ry.a[2] = sin(p); Ry.a[6] = -sin(p); Ry.a[8] = cos(p);
    Rz.a[0] = cos(y); Rz.a[1] = -sin(y); Rz.a[3] = sin(y); Rz.a[4] = cos(y);
    return mul(mul(Rz, Ry), Rx);
}
// Strict numeric attributes: exactly `n` whitespace-separated numbers, nothing else (a malformed
// attribute is an error, never a silent zero or identity).
struct UrdfError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
std::vector<double> nums(const std::string& s, size_t n, const char* what) {
    std::vector<double> v;
    const char* p = s.c_str();
    for (;;) {
        while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') ++p;
        if (!*p) break;
        char* end = nullptr;
        errno = 0;
        const double x = std::strtod(p, &end);
        if (end == p || errno == ERANGE || !std::isfinite(x))
            throw UrdfError(std::string("malformed number in ") + what + "=\"" + s + "\"");
        v.push_back(x);
        p = end;
    }
    if (v.size() != n)
        throw UrdfError(std::string(what) + "=\"" + s + "\" must hold " + std::to_string(n) + " number(s)");
    return v;
}
double num1(const std::string& s, const char* what) { return nums(s, 1, what)[0]; }
void origin(const Xml* o, M3& R, V3& p) {
    R = M3();
    p = V3();
    if (!o) return;
    const auto xyz = nums(o->get("xyz", "0 0 0"), 3, "origin xyz");
    const auto r = nums(o->get("rpy", "0 0 0"), 3, "origin rpy");
    p = V3{{xyz[0], xyz[1], xyz[2]}};
    R = rpy(r[0], r[1], r[2]);
}

struct Inertial {
    double m = 0;
    V3 c;
    M3 I = M3{{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    Inertial transformed(const M3& R, const V3& p) const {
        Inertial o;
        o.m = m;
        o.c = add(mv(R, c), p);
        o.I = mul(mul(R, I), transpose(R));
        return o;
    }
};
Inertial combine(const Inertial& a, const Inertial& b) {
    Inertial o;
    o.m = a.m + b.m;
    if (o.m == 0.0) return Inertial();
    for (int i = 0; i < 3; ++i) o.c.v[i] = (a.m * a.c.v[i] + b.m * b.c.v[i]) / o.m;
    auto shift = [&](const Inertial& x) {
        M3 r;
        double d[3] = {x.c.v[0] - o.c.v[0], x.c.v[1] - o.c.v[1], x.c.v[2] - o.c.v[2]};
        const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) r.a[3 * i + j] = x.I.a[3 * i + j] + x.m * ((i == j ? dd : 0.0) - d[i] * d[j]);
        return r;
    };
    const M3 A = shift(a), B = shift(b);
    for (int k = 0; k < 9; ++k) o.I.a[k] = A.a[k] + B.a[k];
    return o;
}

struct Joint {
    std::string name, type, parent, child;
    M3 R;
    V3 p, axis;
};
struct Frame {
    M3 R;
    V3 p;
};
struct Cluster {
    Inertial inert;
    std::vector<std::pair<std::string, Frame>> out;  // revolute joints leaving the cluster
    std::map<std::string, Frame> frames;             // links rigidly attached (incl. the root)
};

struct Robot {
    std::map<std::string, Inertial> links;
    std::vector<std::string> link_order;
    std::map<std::string, Joint> joints;
    std::vector<std::string> joint_order;
    std::map<std::string, std::vector<std::string>> children;  // link -> joint names (file order)

    Cluster lump(const std::string& link) const {  // tools/gen_model.py build().lump
        Cluster c;
        c.inert = links.at(link);
        c.frames[link] = Frame();
        std::vector<std::tuple<std::string, M3, V3>> stack{{link, M3(), V3()}};
        while (!stack.empty()) {
            auto [lk, R, p] = stack.back();
            stack.pop_back();
            auto it = children.find(lk);
            if (it == children.end()) continue;
            for (const auto& jn : it->second) {
                const Joint& j = joints.at(jn);
                const M3 Rc = mul(R, j.R);
                const V3 pc = add(mv(R, j.p), p);
                if (j.type == "fixed") {
                    c.inert = combine(c.inert, links.at(j.child).transformed(Rc, pc));
                    c.frames[j.child] = Frame{Rc, pc};
                    stack.emplace_back(j.child, Rc, pc);
                } else {
                    c.out.emplace_back(jn, Frame{Rc, pc});
                }
            }
        }
        return c;
    }
};

int32_t err(const std::string& m) {
    wbc_internal_set_error(m.c_str());
    return WBC_ERR_ARG;
}

}  // namespace

static int32_t model_from_urdf(const char* path, const char* const* legs, const char* const* joints,
                               const char* foot_suffix, wbc_model* out) {
    if (!path || !out) return err("wbc_model_from_urdf: null argument");
    std::ifstream f(path);
    if (!f) return err(std::string("wbc_model_from_urdf: cannot open ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    Xml doc;
    std::string perr;
    if (!parse_xml(ss.str(), doc, perr)) return err("wbc_model_from_urdf: " + perr);
    const Xml* robot = doc.child("robot");
    if (!robot) return err("wbc_model_from_urdf: no <robot> element");
    Robot rb;
    for (const auto& el : robot->kids) {
        if (el->name == "link") {
            Inertial in;
            if (const Xml* ie = el->child("inertial")) {
                M3 R;
                V3 p;
                origin(ie->child("origin"), R, p);
                const Xml* m = ie->child("mass");
                const Xml* a = ie->child("inertia");
                if (!m || !a) return err("wbc_model_from_urdf: incomplete <inertial> in link " + el->get("name"));
                in.m = num1(m->get("value", "0"), "mass value");
                if (!(in.m >= 0.0)) return err("wbc_model_from_urdf: negative mass in link " + el->get("name"));
                auto g = [&](const char* k) { return num1(a->get(k, "0"), k); };
                M3 I{{g("ixx"), g("ixy"), g("ixz"), g("ixy"), g("iyy"), g("iyz"), g("ixz"), g("iyz"), g("izz")}};
                in.c = p;
                in.I = mul(mul(R, I), transpose(R));
            }
            rb.links[el->get("name")] = in;
            rb.link_order.push_back(el->get("name"));
        } else if (el->name == "joint") {
            Joint j;
            j.name = el->get("name");
            j.type = el->get("type");
            const Xml* pa = el->child("parent");
            const Xml* ch = el->child("child");
            if (!pa || !ch) return err("wbc_model_from_urdf: joint without parent/child: " + j.name);
            j.parent = pa->get("link");
            j.child = ch->get("link");
            origin(el->child("origin"), j.R, j.p);
            j.axis = V3{{1, 0, 0}};
            if (const Xml* ax = el->child("axis")) {
                const auto v = nums(ax->get("xyz"), 3, "axis xyz");
                const double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                if (!(n > 1e-12)) return err("wbc_model_from_urdf: zero joint axis in " + j.name);
                j.axis = V3{{v[0] / n, v[1] / n, v[2] / n}};  // URDF axes are unit vectors; normalise
            }
            rb.joints[j.name] = j;
            rb.joint_order.push_back(j.name);
            rb.children[j.parent].push_back(j.name);
        }
    }
    // the floating base: the one link that is nobody's child
    std::map<std::string, int> is_child;
    for (const auto& jn : rb.joint_order) is_child[rb.joints[jn].child] = 1;
    std::string base;
    int nroots = 0;
    for (const auto& ln : rb.link_order)
        if (!is_child.count(ln)) { base = ln; ++nroots; }
    if (nroots != 1) return err("wbc_model_from_urdf: expected one root link, found " + std::to_string(nroots));
    for (const auto& jn : rb.joint_order) {
        const auto& t = rb.joints[jn].type;
        if (t != "fixed" && t != "revolute" && t != "continuous")
            return err("wbc_model_from_urdf: unsupported joint type " + t + " (" + jn + ")");
        if (!rb.links.count(rb.joints[jn].child) || !rb.links.count(rb.joints[jn].parent))
            return err("wbc_model_from_urdf: joint " + jn + " references an unknown link");
    }
    static const char* kLegs[4] = {"LH", "LF", "RF", "RH"};  // model order, cpp:81,234,327-341
    static const char* kJoints[3] = {"HAA", "HFE", "KFE"};
    const char* const* L = legs ? legs : kLegs;
    const char* const* J = joints ? joints : kJoints;
    const std::string fs = foot_suffix ? foot_suffix : "FOOT";

    wbc_model m;
    std::memset(&m, 0, sizeof(m));
    const Cluster bc = rb.lump(base);
    m.base_mass = bc.inert.m;
    for (int i = 0; i < 3; ++i) m.base_com[i] = bc.inert.c.v[i];
    for (int k = 0; k < 9; ++k) m.base_inertia[k] = bc.inert.I.a[k];
    double total = bc.inert.m;
    // every moving joint off the base must be a leg's first joint: anything else (an arm, a
    // second chain) would carry mass the lumped 12-DoF model cannot represent
    if (bc.out.size() != 4)
        return err("wbc_model_from_urdf: " + std::to_string(bc.out.size()) +
                   " moving joints leave the base (expected the 4 leg roots)");
    for (int l = 0; l < 4; ++l) {
        std::string jn = std::string(L[l]) + "_" + J[0];
        Frame fr;
        bool found = false;
        for (const auto& o : bc.out)
            if (o.first == jn) { fr = o.second; found = true; }
        if (!found) return err("wbc_model_from_urdf: joint " + jn + " does not leave the base");
        for (int k = 0; k < 3; ++k) {
            const Joint& j = rb.joints[jn];
            if (j.type == "fixed") return err("wbc_model_from_urdf: joint " + jn + " is fixed");
            const Cluster c = rb.lump(j.child);
            wbc_link& lk = m.link[l][k];
            for (int q = 0; q < 9; ++q) lk.R[q] = fr.R.a[q];
            for (int q = 0; q < 3; ++q) { lk.p[q] = fr.p.v[q]; lk.axis[q] = j.axis.v[q]; lk.com[q] = c.inert.c.v[q]; }
            lk.mass = c.inert.m;
            for (int q = 0; q < 9; ++q) lk.inertia[q] = c.inert.I.a[q];
            total += c.inert.m;
            if (k < 2) {
                const std::string nxt = std::string(L[l]) + "_" + J[k + 1];
                int cnt = 0;
                for (const auto& o : c.out)
                    if (o.first == nxt) { fr = o.second; ++cnt; }
                if (cnt != 1) return err("wbc_model_from_urdf: joint " + nxt + " does not follow " + jn);
                if (c.out.size() != 1)
                    return err("wbc_model_from_urdf: link after " + jn + " has " + std::to_string(c.out.size()) +
                               " moving child joints (a leg is one chain)");
                jn = nxt;
            } else {
                if (!c.out.empty()) return err("wbc_model_from_urdf: leg " + std::string(L[l]) + " has more than 3 joints");
                const std::string foot = std::string(L[l]) + "_" + fs;
                auto it = c.frames.find(foot);
                if (it == c.frames.end()) return err("wbc_model_from_urdf: frame " + foot + " not in the last body of its leg");
                for (int q = 0; q < 3; ++q) m.foot[l][q] = it->second.p.v[q];
            }
        }
    }
    m.total_mass = total;  // model_.getTotalMass(), cpp:72
    *out = m;
    return WBC_OK;
}

// No exception crosses the C boundary (wbc.h): malformed numbers and allocation failures become
// WBC_ERR_ARG with the message in wbc_last_error().
extern "C" int32_t wbc_model_from_urdf(const char* path, const char* const* legs, const char* const* joints,
                                       const char* foot_suffix, wbc_model* out) {
    try {
        return model_from_urdf(path, legs, joints, foot_suffix, out);
    } catch (const std::exception& e) {
        return err(std::string("wbc_model_from_urdf: ") + e.what());
    } catch (...) {
        return err("wbc_model_from_urdf: unknown error");
    }
}
