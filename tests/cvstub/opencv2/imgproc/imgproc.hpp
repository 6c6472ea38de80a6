// TEST-ONLY stand-in for <opencv2/imgproc/imgproc.hpp> (apps/demo.cpp includes it and calls nothing
// from it outside comments).  Never used by the product.
#pragma once
#include "../core/core.hpp"
