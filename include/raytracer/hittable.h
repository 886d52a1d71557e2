// hittable.h — name-compatible entry point for code written against the reference's
// programs/hittable.h; the whole host API lives in psrt/rtweekend.hpp.
#pragma once
#include "../psrt/rtweekend.hpp"
