// mrp_env12.hip -- env id 12's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 12
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(12)
