// compile-check stand-in (see opencv2/core/core.hpp)
#pragma once
#include "opencv2/core/core.hpp"
