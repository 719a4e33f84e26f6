// mpc_qp_internal.hpp -- host builder facts used by the device builder (impc_qp.hip), not ABI.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/impc_mpc.h"

// CSC positions (into Ax) of the obstacle-row entries of stage i / obstacle j, in the order the
// reference inserts them (fxx, fyy, fzz, slack: mpcPlanner.cpp:1052-1069) at 4 (i K + j) + e,
// and the first row of the obstacle block.  0 on success.
int impc_mpc_obstacle_layout(const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic,
                             std::vector<int64_t> &slots, int64_t &obs_row_off);
