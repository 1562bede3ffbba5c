// Device helpers shared by the site and guide kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mininf_amd.h"
#include "device_math.hpp"

