// mrp_env15.hip -- env id 15's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 15
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(15)
