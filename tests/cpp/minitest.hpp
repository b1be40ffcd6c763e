// A few doctest-style macros (the reference's tests use doctest, which is not in this image),
// so the C++ tests read like inference/test/t-*.cpp.
#pragma once
#include <cstdio>
#include <exception>
#include <functional>
#include <string>
#include <vector>

namespace minitest {
struct Case { const char* name; std::function<void()> fn; const char* group; };
inline std::vector<Case>& registry() { static std::vector<Case> r; return r; }
inline int& failures() { static int f = 0; return f; }
inline int& checks() { static int c = 0; return c; }
struct Reg {
    Reg(const char* n, const char* g, std::function<void()> f) { registry().push_back({n, std::move(f), g}); }
};
struct Abort {};
inline void fail(const char* file, int line, const std::string& what) {
    ++failures();
    std::printf("  FAILED %s:%d: %s\n", file, line, what.c_str());
}
}  // namespace minitest

#define MT_CAT2(a, b) a##b
#define MT_CAT(a, b) MT_CAT2(a, b)
// TEST_CASE_G(name, group): group "cpu" runs without a GPU, "gpu" needs one.
#define TEST_CASE_G(name, group)                                                              \
    static void MT_CAT(mt_fn_, __LINE__)();                                                   \
    static minitest::Reg MT_CAT(mt_reg_, __LINE__)(name, group, MT_CAT(mt_fn_, __LINE__));    \
    static void MT_CAT(mt_fn_, __LINE__)()
#define CHECK(expr)                                                                           \
    do {                                                                                      \
        ++minitest::checks();                                                                 \
        if (!(expr)) minitest::fail(__FILE__, __LINE__, #expr);                               \
    } while (0)
#define CHECK_FALSE(expr) CHECK(!(expr))
#define REQUIRE(expr)                                                                         \
    do {                                                                                      \
        ++minitest::checks();                                                                 \
        if (!(expr)) { minitest::fail(__FILE__, __LINE__, #expr); throw minitest::Abort{}; }  \
    } while (0)
#define CHECK_THROWS_WITH(expr, msg)                                                          \
    do {                                                                                      \
        ++minitest::checks();                                                                 \
        bool thrown_ = false;                                                                 \
        try { (void)(expr); } catch (const std::exception& e_) {                              \
            thrown_ = true;                                                                   \
            if (std::string(e_.what()) != (msg))                                              \
                minitest::fail(__FILE__, __LINE__, std::string("threw \"") + e_.what() +       \
                                                       "\", expected \"" + (msg) + "\"");     \
        }                                                                                     \
        if (!thrown_) minitest::fail(__FILE__, __LINE__, std::string(#expr) + " did not throw"); \
    } while (0)

#define CHECK_THROWS(expr)                                                                    \
    do {                                                                                      \
        ++minitest::checks();                                                                 \
        bool thrown_ = false;                                                                 \
        try { (void)(expr); } catch (const std::exception&) { thrown_ = true; }               \
        if (!thrown_) minitest::fail(__FILE__, __LINE__, std::string(#expr) + " did not throw"); \
    } while (0)

// main: run the cases of the groups named on the command line (default: all).
#define MINITEST_MAIN(setup)                                                                  \
    int main(int argc, char** argv) {                                                         \
        std::vector<std::string> groups;                                                      \
        setup(argc, argv, groups);                                                            \
        int ran = 0;                                                                          \
        for (auto& c : minitest::registry()) {                                                \
            bool on = groups.empty();                                                         \
            for (auto& g : groups) on = on || g == c.group;                                   \
            if (!on) continue;                                                                \
            ++ran;                                                                            \
            const int before = minitest::failures();                                          \
            std::printf("[ RUN  ] %s\n", c.name);                                             \
            std::fflush(stdout);                                                              \
            try { c.fn(); } catch (const minitest::Abort&) {                                  \
            } catch (const std::exception& e) {                                               \
                minitest::fail(__FILE__, __LINE__, std::string("exception: ") + e.what());    \
            }                                                                                 \
            std::printf("[ %s ] %s\n", minitest::failures() == before ? " OK " : "FAIL", c.name); \
            std::fflush(stdout);                                                              \
        }                                                                                     \
        std::printf("%d cases, %d checks, %d failures\n", ran, minitest::checks(), minitest::failures()); \
        return minitest::failures() == 0 && ran > 0 ? 0 : 1;                                  \
    }
