// Compile-check stand-in for the OpenCV 2.4 surface the ORB-SLAM2 headers and the orbx shims
// (include/compat/) name.  Declarations only: tests/test_compat_compile.py runs the compiler with
// -fsyntax-only, nothing is linked or executed.  Not OpenCV; not used by any product path.
#pragma once
#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>
// OpenCV 2.4's headers leave std names usable unqualified; the ORB-SLAM2 headers rely on it
using namespace std;

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5

namespace cv {
template <class T>
struct Point_ {
  T x, y;
  Point_() : x(0), y(0) {}
  Point_(T a, T b) : x(a), y(b) {}
};
typedef Point_<float> Point2f;
typedef Point_<int> Point2i;
typedef Point2i Point;
template <class T>
struct Point3_ {
  T x, y, z;
};
typedef Point3_<float> Point3f;

struct KeyPoint {
  Point2f pt;
  float size, angle, response;
  int octave, class_id;
};

struct DMatch {
  int queryIdx, trainIdx, imgIdx;
  float distance;
};

struct Range {
  int start, end;
  Range(int a, int b) : start(a), end(b) {}
};

struct Mat {
  int rows = 0, cols = 0;
  size_t step = 0;
  unsigned char* data = nullptr;
  Mat() {}
  Mat(int r, int c, int type);
  Mat clone() const;
  Mat row(int y) const;
  Mat col(int x) const;
  Mat rowRange(int a, int b) const;
  Mat colRange(int a, int b) const;
  Mat t() const;
  Mat inv() const;
  void copyTo(Mat& m) const;
  void create(int r, int c, int type);
  void release();
  bool empty() const;
  double dot(const Mat& m) const;
  template <class T>
  T& at(int i);
  template <class T>
  const T& at(int i) const;
  template <class T>
  T& at(int i, int j);
  template <class T>
  const T& at(int i, int j) const;
  template <class T>
  T* ptr(int i = 0);
  template <class T>
  const T* ptr(int i = 0) const;
};
Mat operator*(const Mat& a, const Mat& b);
Mat operator+(const Mat& a, const Mat& b);
Mat operator-(const Mat& a, const Mat& b);
Mat operator-(const Mat& a);
Mat operator*(double s, const Mat& a);
Mat operator/(const Mat& a, double s);
double norm(const Mat& a);

struct _InputArray {
  _InputArray(const Mat& m);
  Mat getMat() const;
  bool empty() const;
};
struct _OutputArray {
  _OutputArray(Mat& m);
  void release() const;
  void create(int r, int c, int type) const;
  Mat getMat() const;
};
typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;
}  // namespace cv
