// formats.hip — Gaussian PLY files for gfx950 hosts: GaussianModel::loadPly / savePly
// (gaussian_model.cpp:860-1070), which the reference implements with tinyply (third_party/tinyply/tinyply.h).
//
// File layout (what savePly writes through tinyply, tinyply.h:664-703 for the header): an ASCII header
//   ply / format binary_little_endian 1.0 / element vertex P / property float <name> ... / end_header
// then P interleaved records of 17 + 3 Mr float32: x y z nx ny nz f_dc_0..2 f_rest_0..(3Mr-1) opacity
// scale_0..2 rot_0..3 (62 floats = 248 B at SH degree 3). Normals are written as zeros; f_dc / f_rest are stored
// channel-major (features.transpose(1, 2).flatten(1)): f_rest_{c*Mr + k} = features_rest[p][k][c].
//
// MI355X path: the record block moves between host and HBM as ONE contiguous copy and a HIP kernel does the
// (de)interleave and the SH transposes into / out of the six parameter tensors, so the host only parses the header
// and streams bytes. Loading accepts any property order, extra properties and other elements (tinyply requests
// properties by name), and ascii / big-endian / non-float properties through a slower host conversion to float.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "kernels.h"

namespace omr {

namespace {

enum PlyType { PT_I8, PT_U8, PT_I16, PT_U16, PT_I32, PT_U32, PT_F32, PT_F64, PT_BAD };

PlyType ply_type(const std::string& s)
{
    if (s == "char" || s == "int8") return PT_I8;
    if (s == "uchar" || s == "uint8") return PT_U8;
    if (s == "short" || s == "int16") return PT_I16;
    if (s == "ushort" || s == "uint16") return PT_U16;
    if (s == "int" || s == "int32") return PT_I32;
    if (s == "uint" || s == "uint32") return PT_U32;
    if (s == "float" || s == "float32") return PT_F32;
    if (s == "double" || s == "float64") return PT_F64;
    return PT_BAD;
}

int type_size(PlyType t)
{
    static const int sz[] = {1, 1, 2, 2, 4, 4, 4, 8, 0};
    return sz[t];
}

double read_binary(const unsigned char* p, PlyType t, bool big)
{
    unsigned char b[8];
    const int n = type_size(t);
    for (int i = 0; i < n; ++i) b[i] = big ? p[n - 1 - i] : p[i];
    switch (t) {
    case PT_I8: { int8_t v; std::memcpy(&v, b, 1); return v; }
    case PT_U8: { uint8_t v; std::memcpy(&v, b, 1); return v; }
    case PT_I16: { int16_t v; std::memcpy(&v, b, 2); return v; }
    case PT_U16: { uint16_t v; std::memcpy(&v, b, 2); return v; }
    case PT_I32: { int32_t v; std::memcpy(&v, b, 4); return v; }
    case PT_U32: { uint32_t v; std::memcpy(&v, b, 4); return v; }
    case PT_F32: { float v; std::memcpy(&v, b, 4); return v; }
    case PT_F64: { double v; std::memcpy(&v, b, 8); return v; }
    default: return 0.0;
    }
}

struct PlyProp {
    std::string name;
    PlyType type = PT_BAD, list_count = PT_BAD;
    bool is_list = false;
};

struct PlyElement {
    std::string name;
    int64_t count = 0;
    std::vector<PlyProp> props;
};

constexpr int COLS_MAX = 14 + 45;  // columns loadPly requests at SH degree 3 (no normals)

}  // namespace

// columns: x y z | f_dc_0..2 | f_rest_0..3Mr-1 | opacity | scale_0..2 | rot_0..3, as float offsets into a row
struct PlyColumns {
    int col[COLS_MAX];
};

__global__ __launch_bounds__(256) void ply_unpack_kernel(int P, int Mr, const float* rows, int stride, PlyColumns c,
                                                         float* xyz, float* f_dc, float* f_rest, float* opacity,
                                                         float* scaling, float* rotation)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const float* r = rows + (size_t)p * stride;
    const int nr = 3 * Mr;
    for (int k = 0; k < 3; ++k) xyz[3 * (size_t)p + k] = r[c.col[k]];
    for (int k = 0; k < 3; ++k) f_dc[3 * (size_t)p + k] = r[c.col[3 + k]];
    for (int ch = 0; ch < 3; ++ch)  // file column ch*Mr + k -> features_rest[p][k][ch]
        for (int k = 0; k < Mr; ++k) f_rest[(size_t)p * nr + 3 * k + ch] = r[c.col[6 + ch * Mr + k]];
    opacity[p] = r[c.col[6 + nr]];
    for (int k = 0; k < 3; ++k) scaling[3 * (size_t)p + k] = r[c.col[7 + nr + k]];
    for (int k = 0; k < 4; ++k) rotation[4 * (size_t)p + k] = r[c.col[10 + nr + k]];
}

__global__ __launch_bounds__(256) void ply_pack_kernel(int P, int Mr, const float* xyz, const float* f_dc,
                                                       const float* f_rest, const float* opacity,
                                                       const float* scaling, const float* rotation, float* rows)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int nr = 3 * Mr, stride = 17 + nr;
    float* r = rows + (size_t)p * stride;
    for (int k = 0; k < 3; ++k) r[k] = xyz[3 * (size_t)p + k];
    for (int k = 0; k < 3; ++k) r[3 + k] = 0.f;
    for (int k = 0; k < 3; ++k) r[6 + k] = f_dc[3 * (size_t)p + k];
    for (int ch = 0; ch < 3; ++ch)
        for (int k = 0; k < Mr; ++k) r[9 + ch * Mr + k] = f_rest[(size_t)p * nr + 3 * k + ch];
    r[9 + nr] = opacity[p];
    for (int k = 0; k < 3; ++k) r[10 + nr + k] = scaling[3 * (size_t)p + k];
    for (int k = 0; k < 4; ++k) r[13 + nr + k] = rotation[4 * (size_t)p + k];
}

// ---- host side ---------------------------------------------------------------------------------------------------
struct PlyFile {
    std::string path;
    std::vector<PlyElement> elements;
    int format = 0;  // 0 ascii, 1 binary little endian, 2 binary big endian
    size_t data_offset = 0;
    int vertex = -1;
    int Mr = 0;
    PlyColumns cols{};
    std::string error;
};

static bool ply_parse_header(std::ifstream& in, PlyFile& f)
{
    std::string line;
    if (!std::getline(in, line) || (line != "ply" && line != "PLY" && line != "ply\r")) {
        f.error = "not a PLY file: " + f.path;
        return false;
    }
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string tok;
        ss >> tok;
        if (tok == "format") {
            std::string fmt;
            ss >> fmt;
            f.format = fmt == "ascii" ? 0 : fmt == "binary_little_endian" ? 1 : fmt == "binary_big_endian" ? 2 : -1;
            if (f.format < 0) { f.error = "unknown PLY format " + fmt; return false; }
        } else if (tok == "element") {
            PlyElement e;
            ss >> e.name >> e.count;
            f.elements.push_back(e);
        } else if (tok == "property") {
            if (f.elements.empty()) { f.error = "property before element"; return false; }
            PlyProp p;
            std::string t;
            ss >> t;
            if (t == "list") {
                std::string ct, vt;
                ss >> ct >> vt >> p.name;
                p.is_list = true, p.list_count = ply_type(ct), p.type = ply_type(vt);
            } else {
                ss >> p.name;
                p.type = ply_type(t);
            }
            if (p.type == PT_BAD || (p.is_list && p.list_count == PT_BAD)) {
                f.error = "unknown PLY property type in: " + line;
                return false;
            }
            f.elements.back().props.push_back(p);
        } else if (tok == "end_header") {
            f.data_offset = (size_t)in.tellg();
            return true;
        }  // comment / obj_info / blank: ignored
    }
    f.error = "PLY header without end_header";
    return false;
}

static bool ply_columns(PlyFile& f, int max_sh_degree)
{
    for (size_t i = 0; i < f.elements.size(); ++i)
        if (f.elements[i].name == "vertex") f.vertex = (int)i;
    if (f.vertex < 0) { f.error = "PLY file has no vertex element"; return false; }
    const PlyElement& v = f.elements[f.vertex];
    for (const auto& p : v.props)
        if (p.is_list) { f.error = "list property in the vertex element: " + p.name; return false; }
    f.Mr = (max_sh_degree + 1) * (max_sh_degree + 1) - 1;
    std::vector<std::string> names = {"x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2"};
    for (int i = 0; i < 3 * f.Mr; ++i) names.push_back("f_rest_" + std::to_string(i));
    names.push_back("opacity");
    for (int i = 0; i < 3; ++i) names.push_back("scale_" + std::to_string(i));
    for (int i = 0; i < 4; ++i) names.push_back("rot_" + std::to_string(i));
    for (size_t k = 0; k < names.size(); ++k) {
        int found = -1;
        for (size_t j = 0; j < v.props.size(); ++j)
            if (v.props[j].name == names[k]) { found = (int)j; break; }
        if (found < 0) { f.error = "PLY vertex element lacks property " + names[k]; return false; }
        f.cols.col[k] = found;  // property index; turned into a float offset by the reader
    }
    return true;
}

// reads the vertex element as float rows [P][nprops]; returns false on a short / malformed file
static bool ply_read_rows(PlyFile& f, std::vector<float>& rows, int& stride, bool& raw_f32)
{
    std::ifstream in(f.path, std::ios::binary);
    in.seekg((std::streamoff)f.data_offset);
    const PlyElement& v = f.elements[f.vertex];
    const int np = (int)v.props.size();
    bool all_f32 = true;
    for (const auto& p : v.props) all_f32 = all_f32 && p.type == PT_F32;
    // skip the elements before the vertex element
    for (int e = 0; e < f.vertex; ++e) {
        const PlyElement& el = f.elements[e];
        for (int64_t i = 0; i < el.count; ++i) {
            for (const auto& p : el.props) {
                if (f.format == 0) {
                    if (p.is_list) {
                        double n;
                        in >> n;
                        for (int64_t k = 0; k < (int64_t)n; ++k) { double d; in >> d; }
                    } else {
                        double d;
                        in >> d;
                    }
                } else {
                    if (p.is_list) {
                        unsigned char b[8];
                        in.read((char*)b, type_size(p.list_count));
                        const int64_t n = (int64_t)read_binary(b, p.list_count, f.format == 2);
                        in.seekg(n * type_size(p.type), std::ios::cur);
                    } else {
                        in.seekg(type_size(p.type), std::ios::cur);
                    }
                }
            }
        }
        if (!in) { f.error = "truncated PLY element " + el.name; return false; }
    }
    const size_t P = (size_t)v.count;
    stride = np;
    rows.resize(P * (size_t)np);
    raw_f32 = all_f32 && f.format == 1;
    if (raw_f32) {  // the common case: one read of the record block
        in.read(reinterpret_cast<char*>(rows.data()), (std::streamsize)(rows.size() * sizeof(float)));
        if ((size_t)in.gcount() != rows.size() * sizeof(float)) { f.error = "truncated PLY vertex data"; return false; }
        return true;
    }
    if (f.format == 0) {
        for (size_t i = 0; i < rows.size(); ++i) {
            double d;
            if (!(in >> d)) { f.error = "truncated ascii PLY vertex data"; return false; }
            rows[i] = (float)d;
        }
        return true;
    }
    size_t rec = 0;
    for (const auto& p : v.props) rec += type_size(p.type);
    std::vector<unsigned char> buf(rec * P);
    in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)buf.size());
    if ((size_t)in.gcount() != buf.size()) { f.error = "truncated PLY vertex data"; return false; }
    const unsigned char* q = buf.data();
    for (size_t i = 0; i < P; ++i)
        for (int j = 0; j < np; ++j) {
            rows[i * np + j] = (float)read_binary(q, v.props[j].type, f.format == 2);
            q += type_size(v.props[j].type);
        }
    return true;
}

PlyFile* ply_open(const char* path, int max_sh_degree, std::string& err)
{
    auto* f = new PlyFile();
    f->path = path;
    std::ifstream in(path, std::ios::binary);
    if (!in.is_open() || in.fail()) {
        err = std::string("Fail to open ply file at ") + path;  // gaussian_model.cpp:864
        delete f;
        return nullptr;
    }
    if (!ply_parse_header(in, *f) || !ply_columns(*f, max_sh_degree)) {
        err = f->error;
        delete f;
        return nullptr;
    }
    return f;
}

int64_t ply_num_points(const PlyFile* f) { return f->elements[f->vertex].count; }
int ply_rest_coeffs(const PlyFile* f) { return f->Mr; }
void ply_close(PlyFile* f) { delete f; }

bool ply_read(PlyFile* f, float* const params[6], hipStream_t s, std::string& err)
{
    std::vector<float> rows;
    int stride = 0;
    bool raw = false;
    if (!ply_read_rows(*f, rows, stride, raw)) { err = f->error; return false; }
    const int P = (int)ply_num_points(f);
    if (P == 0) return true;
    float* d_rows = nullptr;
    if (hipMalloc(&d_rows, rows.size() * sizeof(float)) != hipSuccess) { err = "hipMalloc failed"; return false; }
    bool ok = hipMemcpyAsync(d_rows, rows.data(), rows.size() * sizeof(float), hipMemcpyHostToDevice, s) == hipSuccess;
    PlyColumns c = f->cols;
    ply_unpack_kernel<<<div_up((uint32_t)P, 256u), 256, 0, s>>>(P, f->Mr, d_rows, stride, c, params[0], params[1],
                                                                 params[2], params[3], params[4], params[5]);
    ok = ok && hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
    (void)hipFree(d_rows);
    if (!ok) err = "PLY upload failed";
    return ok;
}

bool ply_save(const char* path, int P, int Mr, const float* const params[6], hipStream_t s, std::string& err)
{
    const int stride = 17 + 3 * Mr;
    std::vector<float> rows((size_t)P * stride);
    if (P > 0) {
        float* d_rows = nullptr;
        if (hipMalloc(&d_rows, rows.size() * sizeof(float)) != hipSuccess) { err = "hipMalloc failed"; return false; }
        ply_pack_kernel<<<div_up((uint32_t)P, 256u), 256, 0, s>>>(P, Mr, params[0], params[1], params[2], params[3],
                                                                   params[4], params[5], d_rows);
        bool ok = hipGetLastError() == hipSuccess &&
                  hipMemcpyAsync(rows.data(), d_rows, rows.size() * sizeof(float), hipMemcpyDeviceToHost, s) ==
                      hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess;
        (void)hipFree(d_rows);
        if (!ok) { err = "PLY download failed"; return false; }
    }
    std::string h = "ply\nformat binary_little_endian 1.0\nelement vertex " + std::to_string(P) + "\n";
    auto prop = [&h](const std::string& n) { h += "property float " + n + "\n"; };
    for (const char* n : {"x", "y", "z", "nx", "ny", "nz"}) prop(n);
    for (int i = 0; i < 3; ++i) prop("f_dc_" + std::to_string(i));
    for (int i = 0; i < 3 * Mr; ++i) prop("f_rest_" + std::to_string(i));
    prop("opacity");
    for (int i = 0; i < 3; ++i) prop("scale_" + std::to_string(i));
    for (int i = 0; i < 4; ++i) prop("rot_" + std::to_string(i));
    h += "end_header\n";
    FILE* fp = std::fopen(path, "wb");
    if (!fp) { err = std::string("failed to open ") + path; return false; }  // gaussian_model.cpp:1011
    bool ok = std::fwrite(h.data(), 1, h.size(), fp) == h.size();
    if (ok && !rows.empty()) ok = std::fwrite(rows.data(), sizeof(float), rows.size(), fp) == rows.size();
    ok = (std::fclose(fp) == 0) && ok;
    if (!ok) err = std::string("failed to write ") + path;
    return ok;
}

}  // namespace omr
