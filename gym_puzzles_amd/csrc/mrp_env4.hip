// mrp_env4.hip -- env id 4's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 4
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(4)
