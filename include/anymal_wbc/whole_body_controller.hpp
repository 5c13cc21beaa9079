// anymal_wbc/whole_body_controller.hpp — the include path of the reference node
// (src/whole_body_controller_node.cpp:1), forwarding to the MI355X shim.  With include/ on the
// include path, `#include "anymal_wbc/whole_body_controller.hpp"` followed by
// `WholeBodyController wbc; wbc.run();` builds against the engine (include/wbc_controller.hpp).
#ifndef ANYMAL_WBC_WHOLE_BODY_CONTROLLER_HPP_SHIM
#define ANYMAL_WBC_WHOLE_BODY_CONTROLLER_HPP_SHIM
#include "../wbc_controller.hpp"
#endif
