// mrp_env20.hip -- env id 20's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 20
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(20)
