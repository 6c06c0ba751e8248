// TEST DOUBLE -- the enums of the reference's include/mgenGlobals.h the shim names, for the
// protolib-branch build of tests/cpp/compat_shapes (see protokit.h in this directory).
#ifndef _MGEN_GLOBALS
#define _MGEN_GLOBALS
enum Protocol { INVALID_PROTOCOL, UDP, TCP, SINK, SOURCE };
enum { MIN_SIZE = 28, MAX_SIZE = 8192, MSG_LEN_SIZE = 2, TX_BUFFER_SIZE = 8192,
       MAX_FRAG_SIZE = 65535, MIN_FRAG_SIZE = 76 };
enum MessageStatus { MSG_SEND_FAILED, MSG_SEND_BLOCKED, MSG_SEND_OK };
enum LogEventType {
  INVALID_EVENT = 0, RECV_EVENT, RERR_EVENT, SEND_EVENT, LISTEN_EVENT, IGNORE_EVENT, JOIN_EVENT,
  LEAVE_EVENT, START_EVENT, STOP_EVENT, ON_EVENT, ACCEPT_EVENT, DISCONNECT_EVENT, CONNECT_EVENT,
  OFF_EVENT, SHUTDOWN_EVENT, RECONNECT_EVENT
};
#endif
