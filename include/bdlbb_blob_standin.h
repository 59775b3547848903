// bdlbb_blob_standin.h -- minimal stand-in for BDE's bdlbb::Blob.
//
// BDE (bloomberg/bde 4.39.0.0) is not available in this image, so the
// drop-in bmqp::Crc32c is compiled against this stand-in.  It provides exactly
// the members bmqp::Crc32c::calculate(const bdlbb::Blob&, unsigned) uses
// (/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.cpp:47-67):
// numDataBuffers(), buffer(i).data()/size(), lastDataBufferLength().
// A real BlazingMQ build defines BMQCRC_WITH_BDE and uses <bdlbb_blob.h>.
#ifndef INCLUDED_BDLBB_BLOB_STANDIN
#define INCLUDED_BDLBB_BLOB_STANDIN

#include <vector>

namespace BloombergLP {
namespace bdlbb {

class BlobBuffer {
    char* d_data;
    int d_size;

  public:
    BlobBuffer(char* data, int size) : d_data(data), d_size(size) {}
    char* data() const { return d_data; }
    int size() const { return d_size; }
};

class Blob {
    std::vector<BlobBuffer> d_buffers;
    int d_lastDataBufferLength = 0;

  public:
    /// Append `buffer` as a data buffer (all of its bytes are data).
    void appendDataBuffer(const BlobBuffer& buffer)
    {
        d_buffers.push_back(buffer);
        d_lastDataBufferLength = buffer.size();
    }
    /// Trim the data length of the last data buffer (like Blob::setLength).
    void setLastDataBufferLength(int length) { d_lastDataBufferLength = length; }
    int numDataBuffers() const { return static_cast<int>(d_buffers.size()); }
    const BlobBuffer& buffer(int index) const { return d_buffers[index]; }
    int lastDataBufferLength() const { return d_lastDataBufferLength; }
};

}  // namespace bdlbb
}  // namespace BloombergLP

#endif
