// Test double for std_msgs/Float32MultiArray.h (ROS is absent): the member Robot.h uses.
#pragma once
#include <vector>
namespace std_msgs {
struct Float32MultiArray {
    std::vector<float> data;
};
}  // namespace std_msgs
