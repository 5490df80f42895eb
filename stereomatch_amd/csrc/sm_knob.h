// sm_knob.h -- tuning and diagnostic knobs of the library.
//
// A knob is either a schedule parameter that never changes a result (piece length, repair cap,
// segmentation launch schedule, MST tile-phase cap, ...: tests set them to drive every code path
// of the exact engines), a diagnostic that only prints or counts, or the one fault injection the
// MST_PMS forest test needs.  Product builds read knobs ONLY from the table set through the C-ABI
// entry sm_set_knob() (include/stereomst.h), never from the environment, so a stray variable in a
// production environment cannot change what the library does.  Builds with -DSM_DEV (the tools'
// A/B libraries, `make dev`) also read the environment, and only they contain the experiment
// switches (sm_dev_knob: settled A/B paths, timing-only experiments that skip work).
#pragma once

// the knob's value as set through sm_set_knob (SM_DEV builds: else the environment), or nullptr
const char* sm_knob(const char* name);

// integer value of a knob, or dflt when it is unset
int sm_knob_int(const char* name, int dflt);

#ifdef SM_DEV
#include <stdlib.h>
#define sm_dev_knob(name) getenv(name)
#else
// experiment switches and settled A/B paths: compiled out of product builds (their names do not
// even appear in the library)
#define sm_dev_knob(name) ((const char*)nullptr)
#endif
