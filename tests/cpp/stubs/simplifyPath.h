// Test double for slam_ros/simplifyPath.h: the `polar_point` and `line` members the drop-in
// reads (simplifyPath.h:47-79: alfa, r, C_AR, lineInterval). Written for the compile test.
#pragma once
#include <vector>
#include <gsl/gsl_matrix.h>
using namespace std;
class polar_point {
public:
    polar_point() : alfa(0), r(0) {}
    polar_point(double a, double rr) : alfa(a), r(rr) {}
    double alfa;
    double r;
};
class line {
public:
    line() : alfa(0), r(0), C_AR(nullptr) {}
    double alfa;
    double r;
    gsl_matrix* C_AR;
    vector<polar_point> lineInterval;
};
