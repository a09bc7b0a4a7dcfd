// mrp_env18.hip -- env id 18's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 18
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(18)
