// ORBextractor_host.h — the reference's own ORBextractor declared a second time, as
// ORBextractorHost (and its ExtractorNode as ExtractorNodeHost), next to the real class in the
// same translation unit.  ORBextractor_host.cc compiles ORB_SLAM2/src/ORBextractor.cc under
// these names; the GPU shim (ORBextractor_orbx.cc) falls back to it if the device fails, so a
// Tracking thread never sees an error.  Same class layout as ORB_SLAM2/include/ORBextractor.h
// (it is that header, re-included with the two names renamed).
#pragma once
#include "ORBextractor.h"

#pragma push_macro("ORBEXTRACTOR_H")
#undef ORBEXTRACTOR_H
#define ORBextractor ORBextractorHost
#define ExtractorNode ExtractorNodeHost
#include "ORBextractor.h"
#undef ExtractorNode
#undef ORBextractor
#pragma pop_macro("ORBEXTRACTOR_H")
