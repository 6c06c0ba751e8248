// mgenPayload.h -- drop-in MgenPayload / MgenDataItem / MgenFlowCommand
// (reference include/mgenPayload.h:12-136, src/common/mgenPayload.cpp).
//
// These stay on the host by design: a flow sets its DATA payload once
// and the GPU copies those bytes into every record it packs; MGEN_DATA items are parsed on
// the device by mgenx_data_walk (batch) and here (one item at a time).
//   SetPayloadString  hex -> bytes; len = ceil(strlen/2); an odd length reads the NUL as 0;
//                     non-hex characters are 0 (mgenPayload.cpp:24-55, fromHex :127-166)
//   GetPayloadString  bytes -> upper-case hex, new[]'d (:57-73)
//   MgenFlowCommand   the per-flow 2-bit status bitmask (lo half | hi half) (:276-347)
// Difference: buffers are sized by the requested length (the reference's SetPayloadBytes
// sizes a reallocation by the previous length, mgenPayload.cpp:85-88).
#ifndef _MGEN_PAYLOAD
#define _MGEN_PAYLOAD

#include <string.h>

#include "mgenx_proto.h"

class MgenPayload {
 public:
  MgenPayload() : payload_len(0), buffer_len(0), payload_buffer(nullptr) {}
  ~MgenPayload() { delete[] payload_buffer; }

  UINT16 GetLength() { return payload_len; }

  bool SetPayloadString(const char* text) {
    if (text == nullptr) {
      payload_len = 0;
      return true;
    }
    const size_t n = strlen(text);
    const UINT16 len = (UINT16)(n / 2 + n % 2);
    if (!Allocate(len)) return false;
    payload_len = len;
    UINT8* out = (UINT8*)payload_buffer;
    for (size_t i = 0; i < len; i++) {
      const UINT8 hi = (UINT8)fromHex(text[2 * i]);
      const UINT8 lo = (2 * i + 1 < n) ? (UINT8)fromHex(text[2 * i + 1]) : 0;  // the NUL
      out[i] = (UINT8)((hi << 4) | lo);
    }
    return true;
  }
  static char* GetPayloadString(const char* payloadBytes, UINT16 payloadLen) {
    char* text = new char[2u * payloadLen + 1];
    for (unsigned i = 0; i < payloadLen; i++) {
      text[2 * i] = toHex((char)((payloadBytes[i] >> 4) & 0x0f));
      text[2 * i + 1] = toHex((char)(payloadBytes[i] & 0x0f));
    }
    text[2u * payloadLen] = '\0';
    return text;
  }
  bool SetPayloadBytes(char* data, UINT16 size) {
    if (data == nullptr || size == 0) {
      payload_len = 0;
      return true;
    }
    if (!Allocate(size)) return false;
    memcpy(payload_buffer, data, size);
    payload_len = size;
    return true;
  }
  const char* GetPayloadBytes() const { return (const char*)payload_buffer; }
  UINT32* AccessPayloadBuffer() { return payload_buffer; }
  void SetLength(UINT16 length) { payload_len = length; }
  bool Allocate(UINT16 size) {
    if (size <= buffer_len && payload_buffer) return true;
    delete[] payload_buffer;
    payload_buffer = new UINT32[(size + 3u) / 4u + 1u];
    buffer_len = size;
    return true;
  }

 private:
  static char fromHex(char c) {
    if (c >= '0' && c <= '9') return (char)(c - '0');
    if (c >= 'a' && c <= 'f') return (char)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (char)(c - 'A' + 10);
    return 0;
  }
  static char toHex(char v) { return (v >= 0 && v < 16) ? "0123456789ABCDEF"[(int)v] : '?'; }

  UINT16 payload_len;
  UINT16 buffer_len;
  UINT32* payload_buffer;
};

// MGEN_DATA item: | type u8 | len u8 | ... |  (types > 0x0f are MgenAnalytic::Report items)
class MgenDataItem : public ProtoPkt {
 public:
  MgenDataItem(UINT32* bufferPtr = nullptr, unsigned int bufferBytes = 0,
               bool freeOnDestruct = false)
      : ProtoPkt(bufferPtr, bufferBytes, freeOnDestruct) {
    InitFromBuffer();
  }
  ~MgenDataItem() {}

  enum Type { DATA_ITEM_INVALID = 0, DATA_ITEM_FLOW_CMD };

  static Type GetItemType(UINT32* bufferPtr) { return (Type)(((UINT8*)bufferPtr)[0]); }

  // mgenPayload.cpp:214-246: the item is as long as its len byte says (and must fit)
  bool InitFromBuffer(UINT32* bufferPtr = nullptr, unsigned int numBytes = 0,
                      bool freeOnDestruct = false) {
    if (bufferPtr)
      AttachBuffer(bufferPtr, numBytes, freeOnDestruct);
    else
      ProtoPkt::SetLength(0);
    if (GetBuffer() && GetBufferLength() >= OFFSET_LEN) {
      const UINT8 minLength = GetItemLength();
      if (ProtoPkt::InitFromBuffer(minLength)) return true;
      SetType(DATA_ITEM_INVALID);
    }
    if (bufferPtr) DetachBuffer();
    return false;
  }
  Type GetType() const { return (Type)GetUINT8(OFFSET_TYPE); }
  UINT8 GetItemLength() const { return GetUINT8(OFFSET_LEN); }

  // :248-274
  bool InitIntoBuffer(Type type = DATA_ITEM_INVALID, UINT32* bufferPtr = nullptr,
                      unsigned int bufferBytes = 0, bool freeOnDestruct = false) {
    const unsigned minLength = OFFSET_LEN + 1;
    if (bufferPtr) {
      if (bufferBytes < minLength) return false;
      AttachBuffer(bufferPtr, bufferBytes, freeOnDestruct);
    } else if (GetBufferLength() < minLength) {
      return false;
    }
    memset((char*)AccessBuffer(), 0, minLength);
    SetType(type);
    SetItemLength((UINT8)minLength);
    SetLength(minLength);
    return true;
  }
  void SetType(Type type) { SetUINT8(OFFSET_TYPE, (UINT8)type); }
  void SetItemLength(UINT8 len) { SetUINT8(OFFSET_LEN, len); }

 protected:
  enum { OFFSET_TYPE = 0, OFFSET_LEN = OFFSET_TYPE + 1 };
};

class MgenFlowCommand : public MgenDataItem {
 public:
  MgenFlowCommand(UINT32* bufferPtr = nullptr, unsigned int bufferBytes = 0,
                  bool freeOnDestruct = false)
      : MgenDataItem(bufferPtr, bufferBytes, freeOnDestruct) {}
  ~MgenFlowCommand() {}

  enum Status { FLOW_UNCHANGED = 0, FLOW_SUSPEND = 1, FLOW_RESUME = 2, FLOW_RESET = 3 };

  // The item holds two bitmasks of equal size (bit k of the first = status bit 0 of flow
  // k+1, of the second = status bit 1), growing in 4-byte steps so that len = 4 + 4N
  // covers flows up to 16 + 32N (mgenPayload.cpp:276-317).
  bool SetStatus(UINT32 flowId, Status status) {
    const UINT32 need = NeededLength(flowId);
    if (need > GetBufferLength()) return false;
    if (need > GetLength()) {
      char* p = (char*)AccessBuffer();
      const UINT32 oldHalf = (GetLength() - OFFSET_BITS) / 2;
      const UINT32 newHalf = (need - OFFSET_BITS) / 2;
      // move the old second half up, zero the grown tails of both halves
      memmove(p + OFFSET_BITS + newHalf, p + OFFSET_BITS + oldHalf, oldHalf);
      memset(p + OFFSET_BITS + oldHalf, 0, newHalf - oldHalf);
      memset(p + OFFSET_BITS + newHalf + oldHalf, 0, newHalf - oldHalf);
      SetItemLength((UINT8)need);
      SetLength(need);
    }
    SetType(DATA_ITEM_FLOW_CMD);
    const UINT32 k = flowId - 1;
    const UINT8 bit = (UINT8)(0x80 >> (k & 7));
    char* lo = (char*)AccessBuffer(OFFSET_BITS);
    char* hi = lo + (GetLength() - OFFSET_BITS) / 2;
    lo[k >> 3] = (status & 0x01) ? (char)(lo[k >> 3] | bit) : (char)(lo[k >> 3] & ~bit);
    hi[k >> 3] = (status & 0x02) ? (char)(hi[k >> 3] | bit) : (char)(hi[k >> 3] & ~bit);
    return true;
  }
  bool IsSet() const { return (GetLength() > OFFSET_BITS); }
  UINT32 GetMaxFlowId() const {
    const UINT32 len = GetLength();
    return len > OFFSET_BITS ? 8 * (len - OFFSET_BITS) / 2 : 0;
  }
  Status GetStatus(UINT32 flowId) const {
    if (NeededLength(flowId) > GetLength()) return FLOW_UNCHANGED;
    const UINT32 k = flowId - 1;
    const UINT8 bit = (UINT8)(0x80 >> (k & 7));
    const char* lo = GetBuffer(OFFSET_BITS);
    const char* hi = lo + (GetLength() - OFFSET_BITS) / 2;
    return (Status)(((lo[k >> 3] & bit) ? 1 : 0) | ((hi[k >> 3] & bit) ? 2 : 0));
  }
  char* AccessBitmask(unsigned int offset) { return (char*)AccessBuffer(OFFSET_BITS + offset); }
  UINT8 GetMaskLen() const { return (UINT8)(GetItemLength() - OFFSET_BITS); }

 private:
  enum { OFFSET_BITS = OFFSET_LEN + 1 };
  static UINT32 NeededLength(UINT32 flowId) {
    const UINT32 N = (2 * flowId > 16) ? (2 * flowId - 16 - 1) / 32 + 1 : 0;
    return OFFSET_BITS + 2 + N * 4;
  }
};

#endif  // _MGEN_PAYLOAD
