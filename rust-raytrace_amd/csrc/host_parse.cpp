// Scene-file parser for the reference's Rust-like scene grammar.
//
// Behaviour follows serialize.rs:
//   tokenizer   serialize.rs:362-424  ({ } [ ] ( ) : , # // /* */ "..." identifiers numbers)
//   numbers     serialize.rs:407-413  (greedy [A-Za-z0-9_.+-]* run, then f64::from_str)
//   structs     serialize.rs:524-550  (fields in any order, no separators, unknown field =
//                                      error, missing field = error, repeated field: last wins)
//   boxes       serialize.rs:552-565  (Identifier class name, then the class body)
//   functions   serialize.rs:582-593  (name ( arg , arg ... ))
//   vectors     serialize.rs:596-604  ([ elem elem ... ], no separators)
//   u32         serialize.rs:448-469  (round(), negative -> 0, with the reference's warnings)
//   grammar     serialize.rs:606-814
// Lexer errors take priority over parser errors (serialize.rs:436-440).
//
// Deliberate differences (documented in DESIGN.md): an unterminated /* */
// comment is an error here (the reference loops forever at EOF), and
// SkyboxBackground textures are decoded from BMP / binary PPM only
// (host_texture.cpp; the reference's image crate decodes more formats).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <string>

#include "host_scene.hpp"

namespace rtamd {
namespace {

enum class Tok { Ident, Str, Num, LBrace, RBrace, LBracket, RBracket, LParen, RParen, Colon, Comma, End };

const char* tok_name(Tok t) {
    switch (t) {
    case Tok::Ident: return "Identifier"; case Tok::Str: return "String"; case Tok::Num: return "Number";
    case Tok::LBrace: return "LBrace"; case Tok::RBrace: return "RBrace"; case Tok::LBracket: return "LBracket";
    case Tok::RBracket: return "RBracket"; case Tok::LParen: return "LParen"; case Tok::RParen: return "RParen";
    case Tok::Colon: return "Colon"; case Tok::Comma: return "Comma"; case Tok::End: return "end of file";
    }
    return "?";
}

struct Token {
    Tok kind = Tok::End;
    std::string text;
    double num = 0.0;
};

struct ParseError {
    int code;
    std::string msg;
};

// Rust's f64::from_str accepts: [+-]? (digits [. digits?] | . digits) ([eE] [+-]? digits)?
// and [+-]? (inf | infinity | nan) case-insensitively.  No hex floats.
bool rust_f64_from_str(const std::string& s, double& out) {
    size_t i = 0, n = s.size();
    if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
    std::string rest = s.substr(i);
    auto lower = [](std::string x) { for (auto& c : x) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c))); return x; };
    std::string lr = lower(rest);
    if (lr == "inf" || lr == "infinity" || lr == "nan") {
        double v = (lr == "nan") ? std::nan("") : HUGE_VAL;
        out = (s[0] == '-') ? -v : v;
        return true;
    }
    size_t d0 = i;
    while (i < n && std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
    size_t int_digits = i - d0, frac_digits = 0;
    if (i < n && s[i] == '.') {
        ++i;
        size_t f0 = i;
        while (i < n && std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
        frac_digits = i - f0;
    }
    if (int_digits + frac_digits == 0) return false;
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
        size_t e0 = i;
        while (i < n && std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
        if (i == e0) return false;
    }
    if (i != n) return false;
    errno = 0;
    out = std::strtod(s.c_str(), nullptr);   // glibc strtod is correctly rounded, like Rust's parser
    return true;
}

class Lexer {
public:
    explicit Lexer(const std::string& text) : s_(text) {}

    // Location convention of serialize.rs:28-48: row starts at 1, col counts consumed chars.
    int row() const { return row_; }
    int col() const { return col_; }
    const std::optional<ParseError>& error() const { return error_; }

    const Token& peek() {
        if (!has_peek_) { peeked_ = next_token(); has_peek_ = true; tok_row_ = row_; tok_col_ = col_; }
        return peeked_;
    }
    Token take() {
        peek();
        has_peek_ = false;
        return std::move(peeked_);
    }
    int tok_row() { peek(); return tok_row_; }
    int tok_col() { peek(); return tok_col_; }

private:
    int pc() const { return pos_ < s_.size() ? static_cast<unsigned char>(s_[pos_]) : -1; }
    int getc() {
        if (pos_ >= s_.size()) return -1;
        char c = s_[pos_++];
        if (c == '\n') { ++row_; col_ = 0; } else { ++col_; }
        return static_cast<unsigned char>(c);
    }
    void fail(int code, const std::string& m) {
        if (!error_) error_ = ParseError{code, std::to_string(row_) + ":" + std::to_string(col_) + ": " + m};
    }

    Token next_token() {
        Token t;
        for (;;) {
            if (error_) return t;                       // serialize.rs:371
            while (pc() >= 0 && std::isspace(pc())) getc();
            int c = pc();
            if (c < 0) return t;
            switch (c) {
            case '{': getc(); t.kind = Tok::LBrace; return t;
            case '}': getc(); t.kind = Tok::RBrace; return t;
            case '[': getc(); t.kind = Tok::LBracket; return t;
            case ']': getc(); t.kind = Tok::RBracket; return t;
            case '(': getc(); t.kind = Tok::LParen; return t;
            case ')': getc(); t.kind = Tok::RParen; return t;
            case ':': getc(); t.kind = Tok::Colon; return t;
            case ',': getc(); t.kind = Tok::Comma; return t;
            case '#':
                while (pc() >= 0 && pc() != '\n') getc();
                continue;
            case '/': {
                getc();
                int d = getc();
                if (d == '/') {
                    while (pc() >= 0 && pc() != '\n') getc();
                } else if (d == '*') {
                    // serialize.rs:393-397: skip to '*', drop it, and stop only if the NEXT
                    // char (consumed either way) is '/'.  At EOF the reference never stops.
                    for (;;) {
                        while (pc() >= 0 && pc() != '*') getc();
                        if (pc() < 0) { fail(RT_E_PARSE, "unterminated block comment"); return t; }
                        getc();
                        int e = getc();
                        if (e == '/') break;
                        if (e < 0) { fail(RT_E_PARSE, "unterminated block comment"); return t; }
                    }
                } else {
                    fail(RT_E_PARSE, "invalid token");
                    return t;
                }
                continue;
            }
            case '"': {
                getc();
                t.kind = Tok::Str;
                lex_string(t.text);
                return t;
            }
            default: break;
            }
            if (std::isalpha(c) || c == '_') {
                while (pc() >= 0 && (std::isalnum(pc()) || pc() == '_')) t.text.push_back(static_cast<char>(getc()));
                t.kind = Tok::Ident;
                return t;
            }
            if (std::isdigit(c) || c == '.' || c == '-' || c == '+') {
                while (pc() >= 0 && (std::isalnum(pc()) || pc() == '_' || pc() == '.' || pc() == '-' || pc() == '+'))
                    t.text.push_back(static_cast<char>(getc()));
                double v = 0;
                if (!rust_f64_from_str(t.text, v)) { fail(RT_E_PARSE, "invalid number: " + t.text); return Token{}; }
                t.kind = Tok::Num;
                t.num = v;
                return t;
            }
            fail(RT_E_PARSE, "invalid token");
            return t;
        }
    }

    // serialize.rs:299-356 (escapes; an unknown or malformed escape is dropped)
    void lex_string(std::string& out) {
        for (;;) {
            int c = getc();
            if (c < 0 || c == '"') return;
            if (c != '\\') { out.push_back(static_cast<char>(c)); continue; }
            int e = getc();
            switch (e) {
            case 'n': out.push_back('\n'); break;
            case 'r': out.push_back('\r'); break;
            case 't': out.push_back('\t'); break;
            case '\\': out.push_back('\\'); break;
            case '0': out.push_back('\0'); break;
            case '\'': out.push_back('\''); break;
            case '"': out.push_back('"'); break;
            case '\n': while (pc() >= 0 && std::isspace(pc())) getc(); break;
            default: break;   // \x.., \u{..} and unknown escapes: payload not needed by any scene field we load
            }
            if (e < 0) return;
        }
    }

    const std::string& s_;
    size_t pos_ = 0;
    int row_ = 1, col_ = 0;
    Token peeked_;
    bool has_peek_ = false;
    int tok_row_ = 1, tok_col_ = 0;
    std::optional<ParseError> error_;
};

class Parser {
public:
    explicit Parser(Lexer& lx) : lx_(lx) {}

    [[noreturn]] void fail(const std::string& m, int code = RT_E_PARSE) {
        throw ParseError{code, std::to_string(lx_.row()) + ":" + std::to_string(lx_.col()) + ": " + m};
    }

    Token expect(Tok k, const char* desc) {
        const Token& t = lx_.peek();
        if (t.kind == k) return lx_.take();
        if (t.kind == Tok::End) fail(std::string("expected ") + desc + " (end of file)");
        fail(std::string("expected ") + desc + ", not " + tok_name(t.kind) + (t.text.empty() ? "" : "(\"" + t.text + "\")"));
    }
    bool accept(Tok k) {
        if (lx_.peek().kind == k) { lx_.take(); return true; }
        return false;
    }
    void expect_ident(const char* word) {
        const Token& t = lx_.peek();
        if (t.kind == Tok::Ident && t.text == word) { lx_.take(); return; }
        std::string d = std::string("Identifier(\"") + word + "\")";
        if (t.kind == Tok::End) fail("expected " + d + " (end of file)");
        fail("expected " + d + ", not " + tok_name(t.kind));
    }

    double f64() { return expect(Tok::Num, "Number").num; }                 // serialize.rs:444
    int32_t i32() {                                                          // serialize.rs:449-458
        double n = f64();
        if (std::fabs(n - std::trunc(n)) > 0.01) std::fprintf(stderr, "Warning: %g stored as integer\n", n);
        if (std::fabs(n) > 1677215.0) std::fprintf(stderr, "Warning: integer values past ~2^24+1 are not exact\n");
        double r = std::round(n);
        if (std::isnan(r)) return 0;
        if (r >= 2147483647.0) return 2147483647;
        if (r <= -2147483648.0) return -2147483647 - 1;
        return static_cast<int32_t>(r);
    }
    uint32_t u32() {                                                         // serialize.rs:461-469
        int32_t n = i32();
        if (n < 0) { std::fprintf(stderr, "Warning: unsigned integer %d is negative, using 0\n", n); return 0; }
        return static_cast<uint32_t>(n);
    }
    double ang() {                                                           // serialize.rs:476-488
        double n = f64();
        Token u = expect(Tok::Ident, "Identifier");
        if (u.text == "deg") return n * 3.14159265358979323846264338327950288 / 180.0;
        if (u.text == "rad") return n;
        fail("no such class: " + u.text);
    }
    void triple(double out[3]) {                                             // serialize.rs:490-510
        expect(Tok::LParen, "LParen");
        out[0] = f64(); expect(Tok::Comma, "Comma");
        out[1] = f64(); expect(Tok::Comma, "Comma");
        out[2] = f64(); expect(Tok::RParen, "RParen");
    }
    rt_color color() {                                                       // serialize.rs:512-522
        expect_ident("rgb");
        double c[3];
        triple(c);
        return rt_color{c[0], c[1], c[2]};
    }

    // fn_parse_struct!: `{ name: value ... }`; each handler returns false for an unknown name.
    template <class F>
    void structure(F&& field, int n_fields, unsigned& seen) {
        expect(Tok::LBrace, "LBrace");
        seen = 0;
        while (!accept(Tok::RBrace)) {
            Token name = expect(Tok::Ident, "Identifier");
            int idx = field(name.text, /*probe=*/true);
            if (idx < 0) fail("undefined field: " + name.text);
            expect(Tok::Colon, "Colon");
            field(name.text, /*probe=*/false);
            seen |= 1u << idx;
        }
        if (seen != (1u << n_fields) - 1u) fail("missing one or more fields");
    }

    std::string cls() { return expect(Tok::Ident, "Identifier").text; }

    void shape(rt_object& o) {                                               // serialize.rs:606-625
        std::string c = cls();
        unsigned seen;
        if (c == "Sphere") {
            o.shape = RT_SHAPE_SPHERE;
            structure([&](const std::string& f, bool probe) -> int {
                if (f == "center") { if (!probe) triple(o.geom); return 0; }
                if (f == "radius") { if (!probe) o.geom[3] = f64(); return 1; }
                return -1;
            }, 2, seen);
        } else if (c == "Plane") {
            o.shape = RT_SHAPE_PLANE;
            structure([&](const std::string& f, bool probe) -> int {
                if (f == "point") { if (!probe) triple(o.geom); return 0; }
                if (f == "normal") { if (!probe) triple(o.geom + 3); return 1; }
                return -1;
            }, 2, seen);
        } else {
            fail("no such class: " + c);
        }
    }

    void material(rt_object& o) {                                            // serialize.rs:665-709
        std::string c = cls();
        unsigned seen;
        auto common = [&](const std::string& f, bool probe, int base) -> int {
            if (f == "diffuse") { if (!probe) o.diffuse = color(); return base + 0; }
            if (f == "specular") { if (!probe) o.specular = color(); return base + 1; }
            if (f == "exponent") { if (!probe) o.exponent = f64(); return base + 2; }
            if (f == "ambient") { if (!probe) o.ambient = color(); return base + 3; }
            return -1;
        };
        if (c == "PhongMaterial") {
            o.material = RT_MAT_PHONG;
            structure([&](const std::string& f, bool p) { return common(f, p, 0); }, 4, seen);
        } else if (c == "IndirectPhongMaterial") {
            o.material = RT_MAT_INDIRECT_PHONG;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "samples") { if (!p) o.samples = u32(); return 4; }
                return common(f, p, 0);
            }, 5, seen);
        } else if (c == "FresnelMaterial") {
            o.material = RT_MAT_FRESNEL;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "ior") { if (!p) o.ior = f64(); return 4; }
                return common(f, p, 0);
            }, 5, seen);
        } else if (c == "TransparentMaterial") {
            o.material = RT_MAT_TRANSPARENT;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "specular") { if (!p) o.specular = color(); return 0; }
                if (f == "exponent") { if (!p) o.exponent = f64(); return 1; }
                if (f == "ior") { if (!p) o.ior = f64(); return 2; }
                return -1;
            }, 3, seen);
        } else {
            fail("no such class: " + c);
        }
    }

    rt_object object() {                                                     // serialize.rs:711-716
        rt_object o{};
        unsigned seen;
        structure([&](const std::string& f, bool p) -> int {
            if (f == "bounds") { if (!p) shape(o); return 0; }
            if (f == "material") { if (!p) material(o); return 1; }
            return -1;
        }, 2, seen);
        return o;
    }

    void light_model(rt_light& l) {                                          // serialize.rs:725-751
        std::string c = cls();
        unsigned seen;
        if (c == "PointLight") {
            l.kind = RT_LIGHT_POINT;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "location") { if (!p) triple(l.v); return 0; }
                return -1;
            }, 1, seen);
        } else if (c == "DirectionalLight") {
            l.kind = RT_LIGHT_DIRECTIONAL;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "direction") { if (!p) triple(l.v); return 0; }
                return -1;
            }, 1, seen);
        } else if (c == "AreaLight") {
            l.kind = RT_LIGHT_AREA;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "origin") { if (!p) triple(l.v); return 0; }
                if (f == "side1") { if (!p) triple(l.v + 3); return 1; }
                if (f == "side2") { if (!p) triple(l.v + 6); return 2; }
                return -1;
            }, 3, seen);
        } else {
            fail("no such class: " + c);
        }
    }

    rt_light light() {                                                       // serialize.rs:718-723
        rt_light l{};
        unsigned seen;
        structure([&](const std::string& f, bool p) -> int {
            if (f == "model") { if (!p) light_model(l); return 0; }
            if (f == "color") { if (!p) l.color = color(); return 1; }
            return -1;
        }, 2, seen);
        return l;
    }

    // parse_new_spc.or_else(parse_look_at_spc) (serialize.rs:627-646,660): the
    // alternative is tried when `new` fails; a failure after tokens were
    // consumed then fails again in look_at at the current position.
    void simple_camera(rt_camera& cam) {
        try {
            expect_ident("new");
            expect(Tok::LParen, "LParen");
            double pos[3], look[3], up[3];
            triple(pos); expect(Tok::Comma, "Comma");
            triple(look); expect(Tok::Comma, "Comma");
            triple(up); expect(Tok::Comma, "Comma");
            double im = f64();
            expect(Tok::RParen, "RParen");
            camera_simple_new(pos, look, up, im, cam);
        } catch (const ParseError&) {
            if (lx_.error()) throw;
            expect_ident("look_at");
            expect(Tok::LParen, "LParen");
            double focus[3], look[3], up[3];
            triple(focus); expect(Tok::Comma, "Comma");
            triple(look); expect(Tok::Comma, "Comma");
            triple(up); expect(Tok::Comma, "Comma");
            double pov = ang(); expect(Tok::Comma, "Comma");
            double h = f64();
            expect(Tok::RParen, "RParen");
            camera_look_at(focus, look, up, pov, h, cam);
        }
    }

    void camera(rt_camera& cam) {                                            // serialize.rs:648-663
        std::string c = cls();
        if (c == "SimplePerspectiveCamera") {
            simple_camera(cam);
        } else if (c == "DepthOfFieldCamera") {
            expect_ident("new");
            expect(Tok::LParen, "LParen");
            simple_camera(cam);
            expect(Tok::Comma, "Comma");
            double focus = f64(); expect(Tok::Comma, "Comma");
            double aperture = f64(); expect(Tok::Comma, "Comma");
            uint32_t samples = u32();
            expect(Tok::RParen, "RParen");
            cam.kind = RT_CAMERA_DOF;
            cam.focus = focus;
            cam.aperture = aperture;
            cam.samples = samples;
        } else {
            fail("no such class: " + c);
        }
    }

    void background(rt_scene& s) {                                           // serialize.rs:753-796
        std::string c = cls();
        unsigned seen;
        if (c == "SolidColorBackground") {
            s.background_kind = RT_BG_SOLID;
            structure([&](const std::string& f, bool p) -> int {
                if (f == "color") { if (!p) s.background = color(); return 0; }
                return -1;
            }, 1, seen);
        } else if (c == "SkyboxBackground") {                                  // serialize.rs:759-776
            static const char* kFaces[6] = {"px", "nx", "py", "ny", "pz", "nz"};
            structure([&](const std::string& f, bool p) -> int {
                for (int k = 0; k < 6; ++k) {
                    if (f != kFaces[k]) continue;
                    if (!p) {                                                  // load(path)
                        expect_ident("load");
                        expect(Tok::LParen, "LParen");
                        const std::string path = expect(Tok::Str, "String").text;
                        expect(Tok::RParen, "RParen");
                        std::string why;
                        const int rc = load_texture_file(path, s.skybox[k], why);
                        if (rc != RT_OK) fail("error loading texture " + path + ": " + why, rc == RT_E_UNSUPPORTED ? rc : RT_E_PARSE);
                    }
                    return k;
                }
                return -1;
            }, 6, seen);
            s.background_kind = RT_BG_SKYBOX;
        } else {
            fail("no such class: " + c);
        }
    }

    void scene(rt_scene& s) {                                                // serialize.rs:798-814
        unsigned seen;
        structure([&](const std::string& f, bool p) -> int {
            if (f == "objects") {
                if (!p) {
                    s.objects.clear();
                    expect(Tok::LBracket, "LBracket");
                    while (!accept(Tok::RBracket)) s.objects.push_back(object());
                }
                return 0;
            }
            if (f == "lights") {
                if (!p) {
                    s.lights.clear();
                    expect(Tok::LBracket, "LBracket");
                    while (!accept(Tok::RBracket)) s.lights.push_back(light());
                }
                return 1;
            }
            if (f == "camera") { if (!p) camera(s.camera); return 2; }
            if (f == "background") { if (!p) background(s); return 3; }
            if (f == "options") {
                if (!p) {
                    unsigned oseen;
                    structure([&](const std::string& g, bool q) -> int {
                        if (g == "width") { if (!q) s.width = u32(); return 0; }
                        if (g == "height") { if (!q) s.height = u32(); return 1; }
                        if (g == "antialias") { if (!q) s.antialias = u32(); return 2; }
                        return -1;
                    }, 3, oseen);
                }
                return 4;
            }
            return -1;
        }, 5, seen);
    }

private:
    Lexer& lx_;
};

}  // namespace

int parse_scene_text(const std::string& text, rt_scene& out, std::string& err) {
    Lexer lx(text);
    Parser p(lx);
    rt_scene s;
    try {
        p.scene(s);
    } catch (const ParseError& e) {
        if (lx.error()) { err = lx.error()->msg; return lx.error()->code; }   // serialize.rs:437-440
        err = e.msg;
        return e.code;
    }
    if (lx.error()) { err = lx.error()->msg; return lx.error()->code; }
    out = std::move(s);
    return RT_OK;
}

}  // namespace rtamd
