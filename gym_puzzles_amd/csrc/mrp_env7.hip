// mrp_env7.hip -- env id 7's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 7
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(7)
