// TEST INFRASTRUCTURE ONLY: the reference's vendored glm 0.9.6
// (/root/reference/RayTrace/glm, header-only, used unmodified) behind C
// entry points, to pin the oracle's restatements of the glm arithmetic on
// the hot path:
//   ref_glm_dot4      glm::dot(vec4, vec4)            (func_geometric.inl:75-81)
//   ref_glm_ray_dir   perspective(45, 4/3, 0, 100) * vec4(0, 0, 1, 1)
//                     as MainState.cpp:37-39 builds rayDir
//   ref_glm_sphere    the glm vec4 operations of MainState::intersectSphere
//                     (MainState.cpp:300-327) on glm types
// Built by oracle/Makefile with -ffp-contract=off (one rounding per op).
#include <cmath>

#include "glm/glm.hpp"
#include "glm/gtc/matrix_transform.hpp"

extern "C" {

float ref_glm_dot4(const float a[4], const float b[4]) {
    return glm::dot(glm::vec4(a[0], a[1], a[2], a[3]), glm::vec4(b[0], b[1], b[2], b[3]));
}

void ref_glm_ray_dir(float out[4]) {
    glm::mat4 proj = glm::perspective(45.0f, 4.0f / 3.0f, 0.0f, 100.0f);
    glm::vec4 d = proj * glm::vec4(0, 0, 1, 1);
    out[0] = d.x; out[1] = d.y; out[2] = d.z; out[3] = d.w;
}

float ref_glm_sphere(const float o[4], const float d[4], float radius, const float c[4]) {
    const glm::vec4 origin(o[0], o[1], o[2], o[3]), dir(d[0], d[1], d[2], d[3]);
    const glm::vec4 centre(c[0], c[1], c[2], c[3]);
    const glm::vec4 L = centre - origin;
    const float tca = glm::dot(L, dir);
    if (tca < 0) return 0.0f;
    const float d2 = glm::dot(L, L) - tca * tca;
    const float r2 = radius * radius;
    if (d2 > r2) return 0.0f;
    const float thc = std::sqrt(r2 - d2);
    return tca - thc;
}

}  // extern "C"
