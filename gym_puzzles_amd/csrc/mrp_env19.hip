// mrp_env19.hip -- env id 19's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 19
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(19)
