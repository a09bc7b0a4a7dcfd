// mrp_env17.hip -- env id 17's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 17
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(17)
