// TEST DOUBLE -- Mgen's static logging members, as the reference's mgen.cpp:43-83 defines
// them (fprintf, legacy GMT / local timestamps, epoch timestamps).
#include <time.h>

#include "mgen.h"

Mgen::LogFunction Mgen::Log = fprintf;
void (*Mgen::LogTimestamp)(FILE*, const struct timeval&, bool) = Mgen::LogLegacyTimestamp;
void Mgen::SetEpochTimestamp(bool enable) {
  LogTimestamp = enable ? LogEpochTimestamp : LogLegacyTimestamp;
}
void Mgen::LogEpochTimestamp(FILE* f, const struct timeval& t, bool) {
  Log(f, "%lu.%06lu ", (unsigned long)t.tv_sec, (unsigned long)t.tv_usec);
}
void Mgen::LogLegacyTimestamp(FILE* f, const struct timeval& t, bool localTime) {
  time_t secs = t.tv_sec;
  struct tm* p = localTime ? localtime(&secs) : gmtime(&secs);
  Log(f, "%02d:%02d:%02d.%06lu ", p->tm_hour, p->tm_min, p->tm_sec, (unsigned long)(UINT32)t.tv_usec);
}
