// mrp_tables.h -- host construction of EnvTables / EnvParams (see mrp_tables.cpp).
#pragma once
#include "mrp_config.h"

namespace mrp {
bool build_tables(int env_id, EnvTables& t);
void default_params(int env_id, EnvParams& p);
}  // namespace mrp
