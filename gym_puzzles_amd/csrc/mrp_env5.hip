// mrp_env5.hip -- env id 5's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 5
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(5)
