// ref_glm_probe.cpp -- pins the oracle's glm restatement against the reference's OWN vendored glm.
//
// TEST INFRASTRUCTURE.  Compiled by oracle/build_ref.sh against /root/reference/glm (glm 0.9.8.5,
// header-only, vendored in the reference and compiled as-is) into oracle/_ref/glm_probe.  It
// evaluates, with real glm types, exactly the expressions the reference's hot path evaluates:
//   - processInput's camera re-derivation (myApp.cu:1105-1112) from AppData defaults (utils.h:41-74)
//   - VRC sample positions (kernel.cu:53-59) and the modelAux product (kernel.cu:1048-1050, :62)
//   - TEST matrices (kernel.cu:1177-1216) and the per-sample transform chain (kernel.cu:100-115)
//   - the CPU path model matrix (myApp.cu:1406-1409)
//   - plus normalize / cross / lookAt / inverse / rotate on seeded random inputs
// and prints every input and output as C99 hex floats (JSON).  tests/test_oracle_pin.py compares
// the oracle (and the product's host math) against it bit for bit; tests/golden/glm_vectors.json is
// its committed output, so the pin also holds where /root/reference is absent.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>

#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>

static uint64_t rng = 0x5EED1234ULL;
static float frand() {   // splitmix64 -> [-1, 1)
    uint64_t z = (rng += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (float)((double)(z >> 11) / 9007199254740992.0 * 2.0 - 1.0);
}

static std::string hf(float f) { char b[64]; snprintf(b, sizeof b, "\"%a\"", (double)f); return b; }
static std::string v3s(glm::vec3 v) { return "[" + hf(v.x) + "," + hf(v.y) + "," + hf(v.z) + "]"; }
static std::string v4s(glm::vec4 v) { return "[" + hf(v.x) + "," + hf(v.y) + "," + hf(v.z) + "," + hf(v.w) + "]"; }
static std::string m4s(glm::mat4 m) {   // column-major, m[col][row]
    std::string s = "[";
    for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) s += hf(m[c][r]) + (c == 3 && r == 3 ? "" : ",");
    return s + "]";
}

struct Cam { glm::vec3 pos, front, right, up, tlc; };

// utils.h:41-46 + 53-74, then one processInput pass (myApp.cu:1105-1112) with no key pressed
static Cam default_camera(unsigned W, unsigned H, float* rsw_out, float* rsh_out) {
    glm::vec3 cameraPos = glm::vec3(0.0f, 0.0f, 1.0f);
    glm::vec3 cameraFront = glm::normalize(glm::vec3(0.0f, 0.0f, 0.0f) - cameraPos);
    glm::vec3 up = glm::vec3(0.0f, 1.0f, 0.0f);
    glm::vec3 cameraRight = glm::normalize(glm::cross(cameraFront, up));
    glm::vec3 cameraUp = glm::normalize(glm::cross(cameraRight, cameraFront));
    float view_angle = M_PI / 4;
    float real_screen_width = 2 * std::tan(view_angle);
    float real_screen_height = real_screen_width * H / W;
    glm::mat4 rotationMat = glm::mat4(1.0f), translationMat = glm::mat4(1.0f);
    Cam c;
    c.pos = rotationMat * translationMat * glm::vec4(cameraPos, 1.0f);
    c.front = glm::normalize(glm::vec3(0.0f, 0.0f, 0.0f) - c.pos);
    c.right = glm::normalize(glm::cross(cameraUp, c.front));
    c.up = glm::cross(c.front, c.right);
    c.tlc = c.pos + (real_screen_width / 2) * (-c.right) + (c.up * (real_screen_height / 2));
    (void)cameraRight;
    *rsw_out = real_screen_width; *rsh_out = real_screen_height;
    return c;
}

static Cam oblique_camera() {   // utils.h:77-81 applied raw (myApp.cu:1911-1917)
    Cam c;
    c.pos = glm::vec3(0.456607f, 0.693644f, -0.55711);
    c.front = glm::vec3(-0.456606f, -0.693643f, 0.557109f);
    c.right = glm::vec3(-0.19427f, -0.533349f, -0.823285f);
    c.up = glm::vec3(0.868199f, -0.484147f, 0.108777f);
    c.tlc = glm::vec3(1.51908f, 0.742847f, 0.374952f);
    return c;
}

int main() {
    printf("{\n\"glm_version\": %d,\n", GLM_VERSION);
    // ---- primitives on random inputs
    printf("\"prims\": [\n");
    for (int i = 0; i < 64; ++i) {
        glm::vec3 a(frand(), frand(), frand()), b(frand(), frand(), frand());
        glm::vec3 eye = a * 3.0f;
        glm::mat4 la = glm::lookAt(eye, glm::vec3(0.0f), b);
        glm::mat4 inv = glm::inverse(la);
        float ang = frand() * 3.0f;
        glm::mat4 rot = glm::rotate(glm::translate(glm::mat4(1.0f), a), ang, b);
        glm::mat4 sc = glm::scale(rot, b);
        glm::mat4 mm = inv * sc;
        glm::vec4 mv = mm * glm::vec4(a, 1.0f);
        printf(" {\"a\":%s,\"b\":%s,\"ang\":%s,\"normalize_a\":%s,\"cross_ab\":%s,\"lookat\":%s,"
               "\"inverse\":%s,\"rotate\":%s,\"scale\":%s,\"mul\":%s,\"mulv\":%s}%s\n",
               v3s(a).c_str(), v3s(b).c_str(), hf(ang).c_str(), v3s(glm::normalize(a)).c_str(),
               v3s(glm::cross(a, b)).c_str(), m4s(la).c_str(), m4s(inv).c_str(), m4s(rot).c_str(),
               m4s(sc).c_str(), m4s(mm).c_str(), v4s(mv).c_str(), i == 63 ? "" : ",");
    }
    printf("],\n\"frames\": [\n");
    // ---- frame-level expressions
    const unsigned sizes[][3] = {{100, 100, 100}, {64, 48, 64}, {300, 300, 300}, {700, 700, 500}, {1920, 1080, 500}};
    const long long dims[][3] = {{91, 109, 91}, {182, 218, 182}, {512, 512, 512}};
    bool first = true;
    for (auto& sz : sizes) {
        for (int camk = 0; camk < 2; ++camk) {
            unsigned W = sz[0], H = sz[1], S = sz[2];
            float rsw, rsh;
            Cam c = default_camera(W, H, &rsw, &rsh);
            if (camk == 1) c = oblique_camera();
            float viewplane_distance = 2.0f, front_clip_plane = 0.0f;
            float sample_distance = (viewplane_distance - front_clip_plane) / S;
            glm::mat4 modelAux = glm::translate(glm::mat4(1.0f), glm::vec3(0.5f, 0.5f, 0.5f));
            printf("%s {\"W\":%u,\"H\":%u,\"S\":%u,\"camera\":\"%s\",\"rsw\":%s,\"rsh\":%s,\"sd\":%s,"
                   "\"pos\":%s,\"front\":%s,\"right\":%s,\"up\":%s,\"tlc\":%s,\"vrc_points\":[",
                   first ? "" : ",", W, H, S, camk ? "oblique" : "default", hf(rsw).c_str(), hf(rsh).c_str(),
                   hf(sample_distance).c_str(), v3s(c.pos).c_str(), v3s(c.front).c_str(), v3s(c.right).c_str(),
                   v3s(c.up).c_str(), v3s(c.tlc).c_str());
            first = false;
            // kernel.cu:53-59 + :62 at a deterministic set of (x, y, s)
            for (int k = 0; k < 48; ++k) {
                unsigned x = (unsigned)((frand() * 0.5f + 0.5f) * W) % W, y = (unsigned)((frand() * 0.5f + 0.5f) * H) % H;
                unsigned s = (unsigned)((frand() * 0.5f + 0.5f) * S) % S;
                if (k < 4) { x = (k & 1) ? W - 1 : 0; y = (k & 2) ? H - 1 : 0; s = k * (S / 4); }
                int idx = (int)x, idy = (int)y, idz = (int)s;
                glm::vec3 auxPos = c.tlc + idx * rsw / W * c.right + idy * rsh / H * (-c.up) +
                                   (idz * sample_distance + front_clip_plane) * c.front;
                glm::vec3 q = modelAux * glm::vec4(auxPos, 1.0f);
                printf("%s[%u,%u,%u,%s]", k ? "," : "", x, y, s, v3s(q).c_str());
            }
            printf("],\"test\":[");
            // kernel.cu:1177-1216 host matrices, kernel.cu:100-115 per-sample chain
            for (int di = 0; di < 3; ++di) {
                long long d1 = dims[di][0], d2 = dims[di][1], d3 = dims[di][2];
                int longest_dimension = (int)std::max(d1, std::max(d2, d3));
                glm::mat4 modelCam = glm::mat4(1.0f);
                modelCam = glm::translate(modelCam, glm::vec3(-rsw / 2.0f, -rsh / 2.0f, 0.0f));
                modelCam = glm::scale(modelCam, glm::vec3((rsw / W), rsh / H, -viewplane_distance / S));
                glm::mat4 viewCam = glm::lookAt(c.pos, glm::vec3(0.0f, 0.0f, 0.0f), c.up);
                viewCam = glm::inverse(viewCam);
                glm::mat4 toVolumeTransform = glm::mat4(1.0f);
                glm::mat4 tvtranslate1 = glm::translate(glm::mat4(1.0f), glm::vec3(0.5f, 0.5f, 0.5f));
                glm::mat4 scale = glm::scale(glm::mat4(1.0f), glm::vec3(longest_dimension, longest_dimension, longest_dimension));
                glm::mat4 tvtranslate2 = glm::translate(glm::mat4(1.0f),
                    glm::vec3(d1 / 2.0f - longest_dimension / 2.0f, d2 / 2.0f - longest_dimension / 2.0f,
                              d3 / 2.0f - longest_dimension / 2.0f));
                toVolumeTransform = tvtranslate1 * toVolumeTransform;
                toVolumeTransform = scale * toVolumeTransform;
                toVolumeTransform = tvtranslate2 * toVolumeTransform;
                printf("%s{\"dim\":[%lld,%lld,%lld],\"model_cam\":%s,\"inverse_view\":%s,\"to_volume\":%s,\"points\":[",
                       di ? "," : "", d1, d2, d3, m4s(modelCam).c_str(), m4s(viewCam).c_str(), m4s(toVolumeTransform).c_str());
                for (int k = 0; k < 16; ++k) {
                    unsigned x = (unsigned)((frand() * 0.5f + 0.5f) * W) % W, y = (unsigned)((frand() * 0.5f + 0.5f) * H) % H;
                    unsigned s = (unsigned)((frand() * 0.5f + 0.5f) * S) % S;
                    glm::vec3 position = glm::vec3(x, y, s);
                    position = modelCam * glm::vec4(position, 1.0f);
                    position = viewCam * glm::vec4(position, 1.0f);
                    position = toVolumeTransform * glm::vec4(position, 1.0f);
                    printf("%s[%u,%u,%u,%s]", k ? "," : "", x, y, s, v3s(position).c_str());
                }
                printf("]}");
            }
            printf("]}\n");
        }
    }
    // myApp.cu:1406-1409 CPU-path model matrix
    glm::mat4 cpuModel = glm::mat4(1.0f);
    cpuModel = glm::translate(cpuModel, glm::vec3(0.5f, 0.5f, 0.5f));
    cpuModel = glm::rotate(cpuModel, glm::radians(90.0f), glm::vec3(0.0f, 1.0f, 0.0f));
    cpuModel = glm::rotate(cpuModel, glm::radians(90.0f), glm::vec3(-1.0f, 0.0f, 0.0f));
    printf("],\n\"cpu_path_model\": %s\n}\n", m4s(cpuModel).c_str());
    return 0;
}
