// mrp_env9.hip -- env id 9's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 9
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(9)
