// mrp_env22.hip -- env id 22's lane kernels and launch table (see mrp_lane.h, mrp_ops.h).
#define MRP_ENV 22
#include "mrp_lane.h"

MRP_DEFINE_ENV_OPS(22)
