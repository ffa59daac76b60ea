// host_abi.hpp -- host-only pieces of the C ABI shared by engine.hip and host_abi.cpp: the error
// state, the diagnostic overrides of the planner and the plan a handle is built with.
#pragma once
#include <string>

#include "../../include/mpcqp.h"
#include "symbolic.hpp"

namespace mpcqp {
// records msg as the calling thread's mpcqp_last_error() and returns code
int set_error(int code, const std::string& msg);
// waves per instance forced by MPCQP_WAVES (diagnostics; 0: none), the automatic choice
int waves_per_instance();
int auto_waves(const mpcqp_structure* st);
// the plan mpcqp_create builds for a structure (block caps, step kind, waves, layout); false with
// pl.error set if the structure is unsupported
bool plan_for(const mpcqp_structure* st, Plan& pl);
}  // namespace mpcqp
