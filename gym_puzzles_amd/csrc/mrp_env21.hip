// mrp_env21.hip -- env id 21's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 21
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(21)
