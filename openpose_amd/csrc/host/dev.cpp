// dev.cpp -- kernel-variant switch table behind opk_dev_set / opk::dev_switch (common.h).
#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>

#include "../common.h"
#include "opk.h"

namespace opk {

namespace {
std::mutex g_mu;
std::map<std::string, int>& table()
{
    static std::map<std::string, int> t;
    return t;
}
}  // namespace

int dev_switch(const char* key, int dflt)
{
    std::lock_guard<std::mutex> lock(g_mu);
    const auto it = table().find(key);
    return it == table().end() ? dflt : it->second;
}

namespace {
thread_local LaunchLog* t_log = nullptr;
}

void attach_launch_log(LaunchLog* log) { t_log = log; }
LaunchLog* launch_log() { return t_log; }

void note_launch(const char* fmt, ...)
{
    if (!t_log) return;
    char buf[160];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_log->lines.push_back(t_log->layer + "\t" + buf);
}

}  // namespace opk

extern "C" int opk_dev_set(const char* key, int value, int reset)
{
    if (!key) {
        opk::set_error("opk_dev_set: NULL key");
        return 1;
    }
    std::lock_guard<std::mutex> lock(opk::g_mu);
    if (reset)
        opk::table().erase(key);
    else
        opk::table()[key] = value;
    return 0;
}
