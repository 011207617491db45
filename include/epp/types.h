// epp/types.h — small value types of the C++ host API (the reference uses Eigen;
// Eigen is not a dependency of this build).
#pragma once
#include <cmath>
#include <cstddef>
#include <stdexcept>
#include <vector>

namespace epp {

struct Vec3 {
    double x = 0, y = 0, z = 0;
    Vec3() = default;
    Vec3(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
    double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    double& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    Vec3 operator+(const Vec3& o) const { return {x + o.x, y + o.y, z + o.z}; }
    Vec3 operator-(const Vec3& o) const { return {x - o.x, y - o.y, z - o.z}; }
    Vec3 operator*(double s) const { return {x * s, y * s, z * s}; }
    Vec3 operator/(double s) const { return {x / s, y / s, z / s}; }
    // Eigen's norm(): sqrt of the left-to-right sum of squares
    double norm() const { return std::sqrt((x * x + y * y) + z * z); }
};

// Row-major dense matrix (stands in for Eigen::MatrixXd at the API).
struct Matrix {
    std::size_t rows = 0, cols = 0;
    std::vector<double> data;
    Matrix() = default;
    Matrix(std::size_t r, std::size_t c, double v = 0.0) : rows(r), cols(c), data(r * c, v) {}
    double& operator()(std::size_t r, std::size_t c) { return data[r * cols + c]; }
    double operator()(std::size_t r, std::size_t c) const { return data[r * cols + c]; }
    const double* row(std::size_t r) const { return data.data() + r * cols; }
    double* row(std::size_t r) { return data.data() + r * cols; }
};

}  // namespace epp
