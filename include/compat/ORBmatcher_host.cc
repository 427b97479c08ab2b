// ORBmatcher_host.cc — ORB_SLAM2/src/ORBmatcher.cc compiled unchanged as ORBmatcherHost (see
// ORBmatcher_host.h): the host implementation the GPU shim forwards to and falls back on.  Build
// with the reference's flags and -I ORB_SLAM2/src; the reference source is included from where
// it lies, never copied.
#define ORBmatcher ORBmatcherHost
#include "ORBmatcher.cc"
