// TEST DOUBLE -- the members of the reference's class Mgen (include/mgen.h:195-216) that
// the shim's logging members call, for the protolib-branch build of compat_shapes.  The
// static members are defined in mgen_shape.cpp, as the reference defines them in mgen.cpp.
#pragma once
#include <stdio.h>
#include <sys/time.h>

#include "mgenMsg.h"

class Mgen {
 public:
  typedef int (*LogFunction)(FILE*, const char*, ...);
  static LogFunction Log;
  static void (*LogTimestamp)(FILE*, const struct timeval&, bool);
  static void SetEpochTimestamp(bool enable);
  static void LogEpochTimestamp(FILE* filePtr, const struct timeval& theTime, bool localTime);
  static void LogLegacyTimestamp(FILE* filePtr, const struct timeval& theTime, bool localTime);
  FILE* GetLogFile() { return log_file; }
  bool GetLogBinary() { return log_binary; }
  bool GetLocalTime() { return local_time; }
  bool GetLogFlush() { return log_flush; }
  bool GetLogRx() { return log_rx; }
  bool GetLogData() { return log_data; }
  bool GetLogGpsData() { return log_gps_data; }
  bool GetOffsetPending() { return false; }
  void SetLogFile(FILE* f) { log_file = f; }
  void SetLogBinary(bool v) { log_binary = v; }

 private:
  FILE* log_file = NULL;
  bool log_binary = false, local_time = false, log_flush = false, log_rx = true;
  bool log_data = true, log_gps_data = true;
};
