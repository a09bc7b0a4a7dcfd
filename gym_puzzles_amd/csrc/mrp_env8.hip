// mrp_env8.hip -- env id 8's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 8
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(8)
