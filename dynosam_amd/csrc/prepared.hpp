// prepared.hpp — a solver plan built ahead, off the solver handle's thread.
// The module's deferred sliding windows (backend.cpp WindowWorkers) plan
// each window on the builder thread that constructed it, so the solver
// threads only upload the plan and run the LM. Internal to libdynohip (not
// part of the C-ABI).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "../../include/dynohip.h"

namespace dynohip {

struct PreparedPlan;

// The plan of (g, keys, kind) exactly as dynohip_set_values builds it on a
// single-GPU handle; nullptr with rc / err set when planning fails (the
// handle then plans itself and reports the same error).
PreparedPlan* prepare_plan(const dynohip_graph_view& g, const uint64_t* keys, const uint8_t* kind, size_t n, int& rc,
                           std::string& err);
void free_prepared_plan(PreparedPlan* p);

// dynohip_set_values with a plan prepare_plan built from the graph given to
// the handle (dynohip_set_graph) and the same keys and kinds: the handle
// takes it and hands its previous plan back through `p` (freed by the
// caller). p == nullptr, or a handle that keeps its plan (same structure) or
// is partitioned: as dynohip_set_values.
int set_values_prepared(dynohip_solver* s, PreparedPlan* p, const uint64_t* keys, const uint8_t* kind,
                        const double* data, size_t n);

}  // namespace dynohip
