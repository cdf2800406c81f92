// TEST INFRASTRUCTURE ONLY.  C shim over the reference's unmodified
// RayTrace/Cube.cpp (compiled from /root/reference by oracle/Makefile into
// oracle/_ref/libref_cube.so).  It exposes Cube's constructor, scale, rotate,
// translate and getTriangles (Cube.cpp:6-83) so tests can pin the oracle's
// cube packing against the reference's own code.  Nothing here is product.
#include "Cube.h"

#include <cstring>

extern "C" {

// ops: n records of {kind, x, y, z}; kind 0 = scale, 1 = rotate (radians),
// 2 = translate, applied in order to a cube of colour `colour`.
int ref_cube_build(const float* colour, int n_ops, const float* ops,
                   float* out_vertices /* 36*4 */, float* out_colour /* 4 */) {
    glm::vec4 c(colour[0], colour[1], colour[2], colour[3]);
    Cube cube(c);
    for (int i = 0; i < n_ops; ++i) {
        const float* op = ops + 4 * i;
        glm::vec3 v(op[1], op[2], op[3]);
        switch ((int)op[0]) {
        case 0: cube.scale(v); break;
        case 1: cube.rotate(v); break;
        case 2: cube.translate(v); break;
        default: return -1;
        }
    }
    std::vector<glm::vec4> tris = cube.getTriangles();
    if (tris.size() != 36) return -2;
    for (int i = 0; i < 36; ++i) {
        out_vertices[4 * i + 0] = tris[i].x;
        out_vertices[4 * i + 1] = tris[i].y;
        out_vertices[4 * i + 2] = tris[i].z;
        out_vertices[4 * i + 3] = tris[i].w;
    }
    glm::vec4 col = cube.getColour();
    out_colour[0] = col.x;
    out_colour[1] = col.y;
    out_colour[2] = col.z;
    out_colour[3] = col.w;
    return 0;
}

}  // extern "C"
