// mrp_env6.hip -- env id 6's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 6
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(6)
