// overloads.cpp — TEST INFRASTRUCTURE.  Compile-only probe (`make -C oracle overloads`):
// in the reference's own header context (Src/primitive.h, material.h, medium.h) an
// unqualified sqrt/sin/fabs of a float resolves to the C library's double version.
// That fixes the precision of Sphere::solveQuadratic's sqrt (Src/primitive.h:169-171)
// and SphereMesh::Triangulate's sin/cos (Src/primitive.cpp:177-181) in oracle.c and in
// the device code.
#include <type_traits>

#include "material.h"
#include "medium.h"
#include "primitive.h"

static_assert(std::is_same<decltype(sqrt(1.0f)), double>::value, "sqrt(float) is not double here");
static_assert(std::is_same<decltype(sin(1.0f)), double>::value, "sin(float) is not double here");
static_assert(std::is_same<decltype(cos(1.0f)), double>::value, "cos(float) is not double here");
static_assert(std::is_same<decltype(fabs(1.0f)), double>::value, "fabs(float) is not double here");
