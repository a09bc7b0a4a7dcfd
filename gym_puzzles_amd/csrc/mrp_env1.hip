// mrp_env1.hip -- env id 1's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 1
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(1)
