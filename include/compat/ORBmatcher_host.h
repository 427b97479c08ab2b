// ORBmatcher_host.h — the reference's ORBmatcher declared a second time, as ORBmatcherHost, in
// the GPU shim's translation unit (it is ORB_SLAM2/include/ORBmatcher.h re-included with the
// class renamed).  ORBmatcher_host.cc compiles ORB_SLAM2/src/ORBmatcher.cc under that name; the
// shim (ORBmatcher_orbx.cc) forwards the searches the library does not run to it and falls back
// to it when the device fails, so Tracking / LocalMapping / LoopClosing never see an error.
#pragma once
#include "ORBmatcher.h"

#pragma push_macro("ORBMATCHER_H")
#undef ORBMATCHER_H
#define ORBmatcher ORBmatcherHost
#include "ORBmatcher.h"
#undef ORBmatcher
#pragma pop_macro("ORBMATCHER_H")
