// mrp_env2.hip -- env id 2's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 2
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(2)
