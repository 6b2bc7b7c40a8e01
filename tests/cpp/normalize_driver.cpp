// Prints slam_ekf::normalize_radian (slam_ros_amd/host/robot_ekf.hpp) of each argument, to be
// compared with the oracle's restatement of Robot::normalizeRadian (Robot.cpp:62-71).
#include <cstdio>
#include <cstdlib>

#include "robot_ekf.hpp"

int main(int argc, char** argv)
{
    for (int i = 1; i < argc; i++) {
        double r = std::strtod(argv[i], nullptr);
        slam_ekf::normalize_radian(r);
        std::printf("%.17g\n", r);
    }
    return 0;
}
