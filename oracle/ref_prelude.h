/*
 * ref_prelude.h -- TEST INFRASTRUCTURE ONLY.  Force-included (-include) ahead of the
 * reference's own sources when oracle/Makefile compiles them in place under /root/reference.
 * It adds nothing but standard headers the reference forgot and one using-declaration; it is
 * not a stand-in for any header, library or generated file.
 *
 *  - SURVEY H2: include/vptShadeMethods.h:502 uses std::stack without <stack>.
 *  - SURVEY H1: unqualified abs(double) (include/Sphere.h:34, include/pathTracingUtilities.h:20,
 *    include/volumetricBasicFunctions.h:72, include/microFacetUtilities.h:90,98,
 *    include/samplingFunctions.h:223,230) resolves to int abs() on libstdc++ and corrupts the
 *    image; on the author's platform (macOS/libc++) it is the double overload.  Bringing
 *    std::abs into the global namespace selects the double overload, i.e. fabs semantics.
 */
#include <cmath>
#include <cstdlib>
#include <stack>
#include <tuple>
using std::abs;
