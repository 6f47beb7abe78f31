// opts.h -- the library's internal switches: layout choices kept selectable
// for A/B measurements and tests, read where the old
// code read MAMG_* environment variables.
//
// The product library reads no environment.  A switch changes only through
// mamg_set_option (include/mamg.h: a test and tuning hook, not part of the
// preconditioner's parameters), for the whole process.  The diagnosis build
// (make diag, -DMAMG_DIAG=1) also reads the MAMG_* environment variable of a
// switch the call has not set, so A/B scripts and child-process tests can set
// switches before the library loads; its diagnosis-only switches
// (MAMG_K_VARIANT, MAMG_DEBUG_SUMS, ...) are compiled out of the product.
#pragma once

namespace mamg {

// the switch's value (nullptr: unset, the built-in default applies)
const char* opt(const char* name);

// set (value != nullptr) or reset (nullptr) a switch; false for an unknown name
bool set_opt(const char* name, const char* value);

// the switch names, comma-separated
const char* opt_names();

}  // namespace mamg
