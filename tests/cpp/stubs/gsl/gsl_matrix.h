// Test double for <gsl/gsl_matrix.h>: the fields of gsl_matrix that the drop-in reads through
// line::C_AR (slam_ros/simplifyPath.h:75). Compile-test only; GSL itself is absent.
#pragma once
#include <cstddef>
typedef struct {
    size_t size1, size2, tda;
    double* data;
    void* block;
    int owner;
} gsl_matrix;
