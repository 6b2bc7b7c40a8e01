// ros_output.hpp — the far side of the path: what slam_ros/main.cpp
// publishes after every localize (main.cpp:150-174), without ROS types.
//
//   robotPosition (geometry_msgs::Transform, main.cpp:117): translation = (xPos, yPos, thetaPos);
//     rotation carries the pose-uncertainty ellipse, not a quaternion: x = major axis (axii[1]),
//     y = minor axis (axii[0]), z = angle (main.cpp:155-168); w is never written (0 in a
//     value-initialised message)
//   lines (std_msgs::Float32MultiArray, main.cpp:118): Robot::lineIntervals, the world-frame
//     end points of the lines added as landmarks this cycle (Robot.cpp:869-879), published and
//     then cleared (main.cpp:171-174)
//
// Msg is any type with the geometry_msgs::Transform fields (translation.{x,y,z},
// rotation.{x,y,z,w}); a catkin build passes geometry_msgs::Transform itself.
#pragma once

#include <vector>

namespace slam_ekf {

struct TransformMsg {   // geometry_msgs::Transform
    struct { double x = 0, y = 0, z = 0; } translation;
    struct { double x = 0, y = 0, z = 0, w = 0; } rotation;
};

// One publishing cycle after rover.localize(...): fills the robotPosition message, moves the
// cycle's line end points to `lines_out` and clears them on the robot. Returns getEllipse's
// status; on failure the reference publishes uninitialised axes, here the ones getEllipse left.
template <class Robot, class Msg>
bool publish_cycle(Robot& rover, Msg& msg, std::vector<float>& lines_out)
{
    msg.translation.x = rover.xPos;
    msg.translation.y = rover.yPos;
    msg.translation.z = rover.thetaPos;
    float axii[2] = {0.0f, 0.0f};
    float angle = 0.0f;
    const bool ok = rover.getEllipse(axii, angle);
    msg.rotation.x = axii[1];
    msg.rotation.y = axii[0];
    msg.rotation.z = angle;
    lines_out = rover.lineIntervals.data;
    rover.lineIntervals.data.clear();
    return ok;
}

}  // namespace slam_ekf
