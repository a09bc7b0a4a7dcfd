// mrp_env10.hip -- env id 10's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 10
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(10)
