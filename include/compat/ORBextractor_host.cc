// ORBextractor_host.cc — ORB_SLAM2/src/ORBextractor.cc compiled unchanged as ORBextractorHost
// (see ORBextractor_host.h): the host fallback of the GPU shim.  Build it with the reference's
// own flags and include path (-I ORB_SLAM2/src so that the .cc is found); the reference source
// is included from where it lies, never copied.
#define ORBextractor ORBextractorHost
#define ExtractorNode ExtractorNodeHost
#include "ORBextractor.cc"
