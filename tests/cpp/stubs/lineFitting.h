// Test double for slam_ros/lineFitting.h (only its include of simplifyPath.h matters here).
#pragma once
#include "simplifyPath.h"
