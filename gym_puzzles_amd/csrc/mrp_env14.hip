// mrp_env14.hip -- env id 14's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 14
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(14)
