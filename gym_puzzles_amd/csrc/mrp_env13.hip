// mrp_env13.hip -- env id 13's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 13
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(13)
