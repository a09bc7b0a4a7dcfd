// mrp_env0.hip -- env id 0's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 0
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(0)
