// Robot.h — drop-in replacement for slam_ros/Robot.h (HuaiLeiTang/slam_ros, Robot.h:1-77) in the
// catkin package: same include set, same compile-time constants, same class name and public
// members, so slam_ros/main.cpp compiles unchanged. The EKF runs on the MI355X through
// libslam_ekf.so; see robot_ekf.hpp for the member-by-member mapping and INTEGRATION.md for the
// CMakeLists.txt change (Robot.cpp leaves the build; this header is all the host code needs).
#ifndef ROBOT_H_INCLUDED
#define ROBOT_H_INCLUDED

#include <array>
#include <iostream>
#include <vector>

#include "std_msgs/Float32MultiArray.h"

#include "lineFitting.h"
#include "simplifyPath.h"

#include "robot_ekf.hpp"

#define LINESIZE 100
#define SLAMSIZE 203  // = LINESIZE*2+3
#define MAHALANOBIS 0.4
#define LINENOISE 0.03
#define ENCODERNOISE 0.024
#define SIMULATIONOFF true

class Robot : public slam_ekf::BasicRobot<line, std_msgs::Float32MultiArray, LINESIZE> {
public:
    Robot(double x, double y, double theta)
        : slam_ekf::BasicRobot<line, std_msgs::Float32MultiArray, LINESIZE>(x, y, theta)
    {
    }
};

#endif  // ROBOT_H_INCLUDED
