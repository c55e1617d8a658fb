// ono_plan.h — the exchange-plan builders (ono_plan.cpp) for the executor in
// ono_ring.cpp.  Not part of the ABI (the C entry points are in ono_reduce.h).
#pragma once

#include <vector>

#include "ono_internal.h"

namespace ono {

// pull_grads of rank pos for algo ALLREDUCE / HOPS / DIRECT (n >= 2)
int plan_pull_grads(std::vector<ono_plan_step> &out, int algo, int wire, int pos, int n, size_t size, int segments);
// sub-round j of a host-fed HOPS / DIRECT round (sub_elems == 0: the whole bucket)
int plan_pull_grads_sub(std::vector<ono_plan_step> &out, int algo, int wire, int pos, int n, size_t size,
                        size_t sub_elems, size_t j);
size_t plan_sub_elems(size_t sub_elems);                       // the slice per chunk, a multiple of 64
size_t plan_sub_rounds(int n, size_t size, size_t sub_elems);  // how many sub-rounds cover the bucket
// ono_ps_step over RCCL (n >= 2)
int plan_ps_step(std::vector<ono_plan_step> &out, int pos, int n, size_t nparams);
void plan_buffers(int n, size_t size, size_t nparams, uint64_t *counts);

}  // namespace ono
