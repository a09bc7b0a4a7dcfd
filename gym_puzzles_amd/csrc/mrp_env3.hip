// mrp_env3.hip -- env id 3's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 3
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(3)
