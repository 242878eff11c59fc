// C entry points of cr_math.h (the device's correctly rounded atan / sin / cos / tan) for the
// oracle's CR build (oracle/Makefile: lib/liboracle_cr.so): the same C restatement with the
// trigonometric calls the device makes instead of glibc's.
#include "../../ali-fmm-and-ray-tracing_amd/csrc/cr_math.h"

extern "C" {
double oref_cr_atan(double x) { return crm::atan(x); }
double oref_cr_sin(double x) { return crm::sin(x); }
double oref_cr_cos(double x) { return crm::cos(x); }
double oref_cr_tan(double x) { return crm::tan(x); }
}
