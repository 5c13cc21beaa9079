"""CPU: the reference node's entry builds unchanged against the shim.

whole_body_controller_node's main (src/whole_body_controller_node.cpp:1-8) includes
"anymal_wbc/whole_body_controller.hpp" and runs `WholeBodyController wbc; wbc.run();`.  The
program below (written here, the two statements only, no ROS) must compile and link against
include/ and the in-tree libraries: the class is visible in the global namespace and run() exists
(hpp:41, cpp:678-683).  Without a GPU, constructing the controller must fail loudly (no CPU
fallback): the engine throws "no HIP device".
"""
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quadrupedwholebodycontroller_amd")

NODE = r"""
#include "anymal_wbc/whole_body_controller.hpp"
#include <cstdio>
#include <exception>

int main() {
    try {
        WholeBodyController wbc;
        wbc.run();
    } catch (const std::exception& e) {
        std::printf("%s\n", e.what());
        return 7;
    }
    return 0;
}
"""


def test_reference_node_main_builds_against_the_shim():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "node.cpp"), os.path.join(d, "node")
        open(src, "w").write(NODE)
        r = subprocess.run(["g++", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                            "-L", PKG, "-lwbc_controller", "-lwbc_hip", f"-Wl,-rpath,{PKG}"],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        if os.environ.get("HIP_VISIBLE_DEVICES", "") == "" and not os.path.exists("/dev/kfd"):
            run = subprocess.run([exe], capture_output=True, text=True, timeout=120)
            assert run.returncode == 7 and "HIP device" in run.stdout, (run.returncode, run.stdout, run.stderr)
