// driver.cpp — window / batch trigger arithmetic of the reference backend
// (integer, bit-exact):
//   RGBDBackendModule.hpp:120-144  SlidingWindow::check
//   RGBDBackendModule.cc:201-202   full-batch trigger (frame == full_batch_frame - 1)
#include <cstdint>

#include "../../include/dynohip.h"

extern "C" {

void dynohip_sliding_window_init(dynohip_sliding_window* w, int window, int overlap) {
  if (!w) return;
  w->sliding_window = window;
  w->overlap_size = overlap;
  w->previous_trigger_frame = overlap;  // "previous_trigger_frame starts at overlap"
  w->first_frame = -1;
}

// The reference aborts (glog CHECK_GE) on a first frame that does not fit an
// int and on a triggered window that starts before the first frame
// (RGBDBackendModule.hpp:121-124, 139-141); here both return DYNOHIP_EINVAL
// after the same state updates.
int dynohip_sliding_window_check(dynohip_sliding_window* w, uint64_t frame_k, uint64_t* starting_frame,
                                 uint64_t* ending_frame) {
  if (!w) return DYNOHIP_EINVAL;
  if (w->first_frame == -1) {
    w->first_frame = static_cast<int>(frame_k);
    if (w->first_frame < 0) return DYNOHIP_EINVAL;   // CHECK_GE(first_frame, 0)
  }
  const int frame = static_cast<int>(frame_k) - w->first_frame;
  const bool condition = (w->previous_trigger_frame - (frame - w->sliding_window)) == w->overlap_size;
  if (condition) w->previous_trigger_frame = frame;
  if (ending_frame) *ending_frame = frame_k;
  const int starting = static_cast<int>(frame_k) - w->sliding_window;
  if (starting_frame) *starting_frame = static_cast<uint64_t>(starting);
  if (condition && starting < w->first_frame) return DYNOHIP_EINVAL;   // CHECK_GE(starting_frame, first_frame)
  return condition ? 1 : 0;
}

int dynohip_full_batch_trigger(int64_t full_batch_frame, uint64_t frame_k) {
  return (full_batch_frame - 1 == static_cast<int64_t>(frame_k)) ? 1 : 0;
}

}  // extern "C"
