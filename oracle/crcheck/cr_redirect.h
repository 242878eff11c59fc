/* Force-included into the oracle's CR build: trigonometric calls go to cr_shim.cpp. */
#include <math.h>
double oref_cr_atan(double);
double oref_cr_sin(double);
double oref_cr_cos(double);
double oref_cr_tan(double);
#define atan oref_cr_atan
#define sin oref_cr_sin
#define cos oref_cr_cos
#define tan oref_cr_tan
