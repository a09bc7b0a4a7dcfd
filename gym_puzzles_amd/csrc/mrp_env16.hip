// mrp_env16.hip -- env id 16's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 16
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(16)
