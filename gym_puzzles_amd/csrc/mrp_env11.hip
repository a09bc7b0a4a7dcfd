// mrp_env11.hip -- env id 11's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 11
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(11)
