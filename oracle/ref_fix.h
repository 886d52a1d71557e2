/*
 * ORACLE — test infrastructure only. Force-included (g++ -include) ahead of
 * the UNMODIFIED reference sources by oracle/Makefile.
 *
 * random.h:7 computes `(double)rand() / (RAND_MAX + 1)`; with glibc's int
 * RAND_MAX the `+ 1` overflows, random_double() lands in (-1, 0] and
 * random_in_unit_sphere (vec3.h:83-95) never terminates.
 * Making RAND_MAX a double constant here gives random.h:7 its intended value
 * rand()/(RAND_MAX + 1.0) while random.h itself is compiled as shipped.
 */
#include <stdlib.h>
#undef RAND_MAX
#define RAND_MAX 2147483647.0
